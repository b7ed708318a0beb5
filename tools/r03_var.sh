#!/bin/bash
# Round 3: library variants under trajectory_generation_amd/_variants/<v>/ (names given, or all): the fused parity /
# bit-identity tests, then the driver's command (--steps 20) at 2 waves per SIMD, and 200 steps at 2 and 3.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
vs="$*"; [ -z "$vs" ] && vs=$(ls trajectory_generation_amd/_variants/)
for v in $vs; do
  if [ "$v" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or main_py_case or hard_states or full_step" \
    > gpurun_out/r3v_${v}_tests.log 2>&1 || { echo "== $v TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3v_${v}_tests.log | head; exit 1; }
  echo "== $v: $(tail -1 gpurun_out/r3v_${v}_tests.log)"
  for ws in "2 20" "2 20" "2 200" "3 200"; do
    set -- $ws
    TRAJ_FUSED_WAVES=$1 timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $2 \
      > gpurun_out/r3v_${v}_w$1_s$2.json 2> gpurun_out/r3v_${v}.err || { echo "bench $v failed"; tail -5 gpurun_out/r3v_${v}.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r3v_${v}_w$1_s$2.json'));print('  w$1 s$2 VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
