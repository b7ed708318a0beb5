#!/bin/bash
# Round 4: full -m gpu suite, then config 3 (N = 40 mixed, 20 steps after 5) bench + phase profile for the in-tree
# library (full P at capacity 80, zero-column skip in the capacity-80 condensing) and the packed-P variant, then
# the horizon tiers.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/r4_e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_e_tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_e_tests.log | head -30; exit $rc; }
for v in base nofp; do
  if [ "$v" = base ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
  echo "== $v"
  timeout -k 10 200 python tools/phase_profile.py 0 5 20 40 mixed > gpurun_out/r4_e_${v}_phase40.txt 2>&1 || { tail -5 gpurun_out/r4_e_${v}_phase40.txt; exit 1; }
  grep -E "^(kernel|inputs|condense|scale|solve|total|iters|per residual|solve split)|^  (rollout|stage loop|P rows|penalties)" gpurun_out/r4_e_${v}_phase40.txt
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --horizon 40 --kind mixed --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 > gpurun_out/r4_e_${v}_n40.json 2> gpurun_out/r4_e_${v}_n40.err || { tail -5 gpurun_out/r4_e_${v}_n40.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r4_e_${v}_n40.json'));print('  N40 VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),d.get('solver_stats',{}).get('status_hist'))"
done
unset TRAJMPC_LIB
timeout -k 10 300 python tools/r04_tiers.py > gpurun_out/r4_tiers.json 2> gpurun_out/r4_tiers.err; echo "tiers rc=$?"; cat gpurun_out/r4_tiers.json
