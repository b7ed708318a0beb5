#!/bin/bash
# Round 4 baseline on a fresh box: f64 op microbenchmark, GPU tests, phase profile of the fused 20-step
# launch, and the driver's command.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench/mb_f64ops.bin > gpurun_out/r4_mbops.log 2>&1; rc=$?
cat gpurun_out/r4_mbops.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r4_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r4_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/phase_profile.py 0 5 20 > gpurun_out/r4_phase20.txt 2>&1 && cat gpurun_out/r4_phase20.txt &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-knet > gpurun_out/r4_bench.json 2> gpurun_out/r4_bench.err &&
python -c "import json;d=json.load(open('gpurun_out/r4_bench.json'));print('VALUE',round(d['value']),'ms',round(d['ms_per_step'],4),d['roofline']['kernels_ms'],d.get('solver_stats'))"
