#!/bin/bash
# Round 3: capacity-80 (N = 40) fused instances -- the N = 40 parity / bit-identity tests, then config 3
# (4096 mixed refs, N = 40, dt = 0.05, 20 steps) with the one-wave-per-SIMD instance (1) and the lean
# two-wave instance (2).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fused or per_step_parity or hard_states" > gpurun_out/r3n_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3n_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3n_tests.log | head -20; exit $rc; }
for wv in 1 2; do
  TRAJ_FUSED_WAVES=$wv timeout -k 10 300 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 \
    --horizon 40 --kind mixed --steps ${N40_STEPS:-20} > gpurun_out/r3n_b$wv.json 2> gpurun_out/r3n_b$wv.err || { tail -5 gpurun_out/r3n_b$wv.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3n_b$wv.json'));print('waves $wv VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2), d['solver_stats']['status_hist'])"
done
