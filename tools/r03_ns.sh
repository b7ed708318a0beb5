#!/bin/bash
# 3-wave instance with 3 of the 5 iterate rows parked in LDS (12,776 B: 12 workgroups per CU?) against the
# 5-row build (_variants/ns5): fused bit-identity / parity tests, then W3 at 20 and 200 steps, W2 at 20, and a
# kernel trace of the W3 launch (its grid = the resident slots).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
O=gpurun_out/ns; mkdir -p $O
for v in head ns5; do
  if [ "$v" = head ]; then unset TRAJMPC_LIB; else export TRAJMPC_LIB="$PWD/trajectory_generation_amd/_variants/$v/libtrajmpc.so"; fi
  timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "fused or per_step_parity or main_py_case or hard_states or full_step" \
    > $O/${v}_tests.log 2>&1 || { echo "== $v TESTS FAILED"; grep -E "FAILED|Error|assert" $O/${v}_tests.log | head; exit 1; }
  echo "== $v: $(tail -1 $O/${v}_tests.log)"
  for ws in "3 20" "2 20" "3 20" "3 200" "2 200"; do
    set -- $ws
    TRAJ_FUSED_WAVES=$1 timeout -k 10 200 python bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps $2 \
      > $O/${v}_w$1_s$2.json 2> $O/${v}.err || { echo "bench $v failed"; tail -5 $O/${v}.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${v}_w$1_s$2.json'));print('  w$1 s$2 VALUE',round(d['value']),'kernel_ms',round(d['roofline']['kernel_ms'],3),'iters',round(d['solver_stats']['iters_mean'],2))"
  done
done
unset TRAJMPC_LIB
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
TRAJ_FUSED_WAVES=3 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $PWD/$O/trace -- python3 bench.py --no-cpu --no-knet --no-config1 --no-cold --dataset-steps 0 --steps 20 > $O/trace.log 2>&1
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/ns/trace/**/*kernel_trace.csv", recursive=True):
    g = {}
    for r in csv.DictReader(open(f)):
        if "solve_kernel" in r["Kernel_Name"]:
            k = (r["Kernel_Name"][:48], r.get("Grid_Size_X") or r.get("Grid_Size"), r.get("Workgroup_Size_X") or r.get("Workgroup_Size"), r.get("LDS_Block_Size") or r.get("Lds_Size"))
            g[k] = g.get(k, 0) + 1
    for k, v in g.items(): print("dispatch", k, v)
PY
