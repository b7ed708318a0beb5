#!/bin/bash
# Round-2 GPU measurement at the driver's command (bench.py --steps 20 --warmup 5): parity tests, PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE separately), SQ f64 pass, the bench line, kernel-trace stats of
# the same command, the 20- and 200-step item timelines.  Every GPU step has its own limit; && chain.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
B="python3 bench.py --steps 20 --warmup 5"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
echo tests ok && tail -1 gpurun_out/gpu_tests.log &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- $B --no-cpu --no-knet --dataset-steps 0 > gpurun_out/prof_fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- $B --no-cpu --no-knet --dataset-steps 0 > gpurun_out/prof_write.log 2>&1 &&
python3 tools/pmc_traffic.py --fetch gpurun_out/prof_fetch --write gpurun_out/prof_write --batch 4096 --horizon 20 --fused-steps 20 --out gpurun_out/traffic_r02.json > /dev/null &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAVES -d gpurun_out/pmc_f64 -o run --output-format csv -- $B --no-cpu --no-knet --dataset-steps 0 > gpurun_out/pmc_f64.log 2>&1 &&
python3 tools/pmc_f64.py gpurun_out/pmc_f64 --batch 4096 --steps-per-launch 20 --out gpurun_out/sq_f64_r02.json > /dev/null &&
echo pmc ok &&
timeout -k 10 300 $B --traffic-json gpurun_out/traffic_r02.json --issue-json gpurun_out/sq_f64_r02.json > gpurun_out/bench.json 2> gpurun_out/bench.err &&
echo bench ok &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- $B --no-cpu > gpurun_out/prof_kt.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/prof_kt/run_kernel_trace.csv "solve_kernel<40, true, true>" gpurun_out/solve_dispatches.json > /dev/null &&
echo trace ok &&
timeout -k 10 120 python3 tools/item_timeline.py 20 5 > gpurun_out/tl20.json 2> gpurun_out/tl20.err &&
timeout -k 10 120 python3 tools/item_timeline.py 200 5 > gpurun_out/tl200.json 2> gpurun_out/tl200.err &&
echo all ok
