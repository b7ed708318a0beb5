#!/bin/bash
# KalmanNet on the GPU box: parity tests, the knet bench leg, and a rocprofv3 kernel summary of it.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_knet_gpu.py -x -q -p no:cacheprovider ${KTESTS:+-k "$KTESTS"} > gpurun_out/k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/k_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/knet_bench.py > gpurun_out/k_bench.json 2> gpurun_out/k_bench.err && cat gpurun_out/k_bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o kprof -- python3 tools/knet_bench.py > gpurun_out/k_prof.log 2>&1 &&
find gpurun_out/kprof -name '*kernel_stats.csv' -exec head -25 {} \;
