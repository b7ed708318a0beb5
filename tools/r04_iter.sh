#!/bin/bash
# Round 4 iteration on the GPU box: the -m gpu suite (or the subset in TESTS), the phase profile of the fused
# 20-step launch, and the bench at the driver's command (20 steps) and over 200 steps, for the in-tree library
# and every variant named in VARIANTS (trajectory_generation_amd/_variants/<v>/libtrajmpc.so).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
tag=${TAG:-it}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    ${TESTS:+-k "$TESTS"} > gpurun_out/r4_${tag}_tests.log 2>&1; rc=$?
  tail -2 gpurun_out/r4_${tag}_tests.log
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_${tag}_tests.log | head -30; exit $rc; }
fi
for v in base $VARIANTS; do
  if [ "$v" = base ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
  echo "== $v"
  timeout -k 10 120 python tools/phase_profile.py 0 5 20 > gpurun_out/r4_${tag}_${v}_phase.txt 2>&1 || { tail -5 gpurun_out/r4_${tag}_${v}_phase.txt; exit 1; }
  grep -E "^(kernel|inputs|condense|scale|solve|total|iters|per residual|solve split)|^  (rollout|jac|stage loop|P rows|penalties)" gpurun_out/r4_${tag}_${v}_phase.txt
  for s in ${STEPS:-20 200}; do
    timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $s > gpurun_out/r4_${tag}_${v}_b$s.json 2> gpurun_out/r4_${tag}_${v}_b$s.err || { echo "bench $v $s failed"; tail -5 gpurun_out/r4_${tag}_${v}_b$s.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r4_${tag}_${v}_b$s.json'));print('   steps=$s VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],4),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
