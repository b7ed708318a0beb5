#!/bin/bash
# Linearization rework: MPC GPU parity tests, then the bench at the driver's command and 200 steps, and
# the phase profile.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/lin_tests.log 2>&1; rc=$?
tail -3 gpurun_out/lin_tests.log
[ $rc -eq 0 ] || exit $rc
for s in 20 20 200; do
  timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps $s --warmup 5 > gpurun_out/lin_b.json 2> gpurun_out/lin_b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/lin_b.json'));print($s, 'VALUE', round(d['value']), 'ms/step', round(d['ms_per_step'],4), 'iters', round(d['solver_stats']['iters_mean'],2))"
done
timeout -k 10 120 python tools/phase_profile.py 0 5 20 > gpurun_out/lin_phase.log 2>&1; cat gpurun_out/lin_phase.log | head -22
