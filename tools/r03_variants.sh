#!/bin/bash
# Round 3: for every library build under trajectory_generation_amd/_variants/*/ (or the names given), the fused
# closed-loop bit-identity / parity tests, then the bench at the driver's command (--steps 20) and at 200 steps
# (MPC only).  Results: gpurun_out/r3v_<variant>_*.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
vs="$*"; [ -z "$vs" ] && vs=$(ls trajectory_generation_amd/_variants/)
for v in $vs; do
  export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or main_py_case or hard_states or full_step" \
    > gpurun_out/r3v_${v}_tests.log 2>&1 || { echo "== $v TESTS FAILED"; tail -30 gpurun_out/r3v_${v}_tests.log; exit 1; }
  echo "== $v: $(tail -1 gpurun_out/r3v_${v}_tests.log)"
  for s in 20 200; do
    timeout -k 10 200 python bench.py --no-cpu --no-knet --dataset-steps 0 --steps $s > gpurun_out/r3v_${v}_b$s.json 2> gpurun_out/r3v_${v}_b$s.err || { echo "bench $v $s failed"; tail -5 gpurun_out/r3v_${v}_b$s.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r3v_${v}_b$s.json'));print('   steps=$s VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],4),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
