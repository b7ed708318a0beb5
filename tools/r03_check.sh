#!/bin/bash
# Round 3 check on the GPU box: the whole -m gpu suite, then the MPC bench at the driver's command (20 steps)
# and at 200 steps (MPC only), with the in-tree library.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r3c_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3c_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3c_tests.log | head -20; exit $rc; }
for s in 20 200; do
  timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps $s > gpurun_out/r3c_b$s.json 2> gpurun_out/r3c_b$s.err || { tail -5 gpurun_out/r3c_b$s.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r3c_b$s.json'));print('steps=$s VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],4),'iters',round(d['solver_stats']['iters_mean'],2), d['solver_stats']['status_hist'])"
done
