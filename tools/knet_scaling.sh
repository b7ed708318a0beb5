#!/bin/bash
# per-kernel time of the fused KalmanNet step vs batch size
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kscale -o ks -- python3 tools/knet_scaling.py "$@" > gpurun_out/kscale.log 2>&1 && grep "B=" gpurun_out/kscale.log &&
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/kscale/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "knet_front" in k or "knet_back" in k or "knet_fc2" in k:
        name = "front" if "front" in k else ("back" if "back" in k else "fc2")
        d[(name, int(r["Grid_Size_X"]) if "Grid_Size_X" in r else int(r.get("Grid_Size", 0)))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, g), v in sorted(d.items()):
    v = sorted(v)
    print(f"{name:6s} grid {g:8d}: median {v[len(v)//2]:.1f} us  n={len(v)}")
PY
