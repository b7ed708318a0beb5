#!/bin/bash
# One-wave pipelined sweep variants (TGMPC_PIPE1): fused bit-identity / parity tests per variant, then the
# driver's command (MPC only, 20 timed steps) interleaved over the variants, 3 reps, and 200 steps once.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/pipe1; mkdir -p $O
for v in "$@"; do
  [ "$v" = base ] && continue
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or main_py_case or hard_states or full_step" \
    > $O/${v}_tests.log 2>&1 || { echo "== $v TESTS FAILED"; tail -30 $O/${v}_tests.log; exit 1; }
  echo "== $v: $(tail -1 $O/${v}_tests.log)"
done
for s in 20 20 20 200; do
  for v in "$@"; do
    export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
    timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $s > $O/${v}_$s.json 2> $O/${v}.err || { tail -5 $O/${v}.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_$s.json'));print('$v steps=$s VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],4))"
  done
done
