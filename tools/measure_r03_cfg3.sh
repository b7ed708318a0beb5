#!/bin/bash
# Round-3 config-3 measurement (BASELINE.json configs[2]: 4096 mixed sinusoid / parabola refs, N = 40, dt = 0.05;
# 20 timed steps after 5): PMC traffic (FETCH_SIZE, WRITE_SIZE), the SQ f64 pass, the bench line carrying both,
# kernel-trace dispatches (code-object VGPR / AGPR / LDS / scratch of solve_kernel<80, true, true>), the phase profile.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 20 --warmup 5 --horizon 40 --kind mixed"
M="--no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r3n40_fetch -o run --output-format csv -- $B $M > gpurun_out/r3n40_fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r3n40_write -o run --output-format csv -- $B $M > gpurun_out/r3n40_write.log 2>&1 &&
python3 tools/pmc_traffic.py --fetch gpurun_out/r3n40_fetch --write gpurun_out/r3n40_write --batch 4096 --horizon 40 --fused-steps 20 --out gpurun_out/traffic_r03_n40.json > /dev/null &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d gpurun_out/r3n40_f64 -o run --output-format csv -- $B $M > gpurun_out/r3n40_f64.log 2>&1 &&
python3 tools/pmc_f64.py gpurun_out/r3n40_f64 --batch 4096 --steps-per-launch 20 --horizon 40 --out gpurun_out/sq_f64_r03_n40.json > /dev/null &&
echo pmc ok &&
timeout -k 10 300 $B --no-knet --no-config1 --cpu-traj 512 --cpu-steps 16 --dataset-steps 0 --traffic-json gpurun_out/traffic_r03_n40.json --issue-json gpurun_out/sq_f64_r03_n40.json > gpurun_out/r03_bench_n40_mixed.json 2> gpurun_out/r03_bench_n40_mixed.err &&
python3 -c "import json;d=json.load(open('gpurun_out/r03_bench_n40_mixed.json'));print('N40 VALUE',round(d['value']),'traffic',d['roofline']['traffic'],'issue',d['roofline']['issue'] and round(d['roofline']['issue']['simd_valu_busy_frac'],3))" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n40_kt -o run --output-format csv -- $B $M > gpurun_out/r3n40_kt.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/r3n40_kt/run_kernel_trace.csv "solve_kernel<80, true, true" gpurun_out/r03_solve_dispatches_n40.json > /dev/null &&
timeout -k 10 200 python3 tools/phase_profile.py 0 5 20 40 mixed > gpurun_out/r03_phase20_n40.txt 2>&1 &&
echo cfg3 ok
