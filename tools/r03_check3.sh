#!/bin/bash
# Round 3: the whole -m gpu suite, then the driver's command twice and 200 steps (MPC only; 2 and 3 waves per SIMD).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r3c3_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3c3_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3c3_tests.log | head -20; exit $rc; }
for ws in "0 20" "0 20" "2 200" "3 200"; do
  set -- $ws
  TRAJ_FUSED_WAVES=$1 timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $2 \
    > gpurun_out/r3c3_w$1_s$2.json 2> gpurun_out/r3c3.err || { tail -5 gpurun_out/r3c3.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3c3_w$1_s$2.json'));print('w$1 s$2 VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2), d['solver_stats']['status_hist'])"
done
