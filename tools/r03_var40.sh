#!/bin/bash
# Config 3 (N = 40 mixed, 20 steps) for library variants under trajectory_generation_amd/_variants/<v>/ against
# the in-tree build, alternating: the fused N = 40 tests per variant first.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/v40; mkdir -p $O
for v in "$@"; do
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or hard_states" > $O/${v}_tests.log 2>&1 || { echo "$v TESTS FAILED"; grep -E "FAILED|Error|assert" $O/${v}_tests.log | head; exit 1; }
  echo "== $v: $(tail -1 $O/${v}_tests.log)"
done
for rep in 1 2; do
  for v in head "$@"; do
    if [ "$v" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
    timeout -k 10 300 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --horizon 40 --kind mixed \
      --steps 20 > $O/${v}_$rep.json 2> $O/${v}.err || { tail -5 $O/${v}.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_$rep.json'));print('$v rep $rep VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
