#!/bin/bash
# Round-4 GPU measurement at the driver's command (bench.py --steps 20 --warmup 5): PMC traffic passes (FETCH_SIZE,
# WRITE_SIZE separately), the SQ f64 pass, kernel-trace stats of the bench command and its solve dispatches, the
# phase profile and the 20-step item timeline.  Every GPU step has its own limit; && chain.  Outputs gpurun_out/r4m_*.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 20 --warmup 5"
M="--no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4m_fetch -o run --output-format csv -- $B $M > gpurun_out/r4m_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r4m_write -o run --output-format csv -- $B $M > gpurun_out/r4m_write.log 2>&1 &&
python3 tools/pmc_traffic.py --fetch gpurun_out/r4m_fetch --write gpurun_out/r4m_write --batch 4096 --horizon 20 --fused-steps 20 --out gpurun_out/traffic_r04.json > /dev/null &&
echo traffic ok &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d gpurun_out/r4m_f64 -o run --output-format csv -- $B $M > gpurun_out/r4m_f64.log 2>&1 &&
python3 tools/pmc_f64.py gpurun_out/r4m_f64 --batch 4096 --steps-per-launch 20 --out gpurun_out/sq_f64_r04.json > /dev/null &&
echo sq ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4m_kt -o run --output-format csv -- $B > gpurun_out/r4m_kt.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/r4m_kt/run_kernel_trace.csv "solve_kernel<40, true, true" gpurun_out/r04_solve_dispatches.json > /dev/null &&
echo trace ok &&
timeout -k 10 120 python3 tools/phase_profile.py 0 5 20 > gpurun_out/r04_phase20.txt 2>&1 &&
echo all ok
