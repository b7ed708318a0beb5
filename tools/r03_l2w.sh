#!/bin/bash
# Config 3 (N = 40 mixed, 20 steps): library variants under trajectory_generation_amd/_variants/<v>/ run with the
# lean two-wave capacity-80 instance forced (TRAJ_FUSED_WAVES=2), against the in-tree build's default instance.
# The fused N = 40 tests per variant first (they include both capacity-80 instances' bit-identity).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/l2w; mkdir -p $O
for v in "$@"; do
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or hard_states" > $O/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; grep -E "FAILED|Error|assert" $O/${v}_tests.log | head; exit 1; }
  echo "== $v: $(tail -1 $O/${v}_tests.log)"
done
for rep in 1 2; do
  for v in head "$@"; do
    if [ "$v" = head ]; then unset TRAJMPC_LIB TRAJ_FUSED_WAVES; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so" TRAJ_FUSED_WAVES=2; fi
    timeout -k 10 300 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --horizon 40 --kind mixed \
      --steps 20 > $O/${v}_$rep.json 2> $O/${v}.err || { tail -5 $O/${v}.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v rep $rep VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
