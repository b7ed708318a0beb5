#!/bin/bash
# L2 hit/miss of the KalmanNet kernels (one PMC pass over tools/knet_bench.py, no CPU leg).
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_kl2 -o run --output-format csv -- python3 tools/knet_bench.py > gpurun_out/pmc_kl2.log 2>&1 &&
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_kl2/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"]
    if "knet_" not in k: continue
    name = k.split("::")[1].split("(")[0]
    acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(name, r["Counter_Name"])] += 1
for name, cs in acc.items():
    v = {c: round(x / n[(name, c)]) for c, x in cs.items()}
    h, m = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
    print(name, v, "hit rate %.3f" % (h / max(1, h + m)))
PY
