#!/bin/bash
# Round-1 GPU measurement: parity tests, bench line, kernel-trace stats, PMC traffic passes.
# Every GPU step has its own time limit; steps are chained with && (stop at the first failure).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_kt -o run --output-format csv -- python3 bench.py --no-cpu > gpurun_out/prof_kt.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-knet > gpurun_out/prof_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write -o run --output-format csv -- python3 bench.py --no-cpu --no-knet > gpurun_out/prof_write.log 2>&1 &&
python3 tools/trace_dispatches.py gpurun_out/prof_kt/run_kernel_trace.csv "solve_kernel<40, true, true>" gpurun_out/solve_dispatches.json > /dev/null
