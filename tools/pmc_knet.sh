#!/bin/bash
# PMC passes over the KalmanNet bench leg (tools/knet_bench.py): SQ issue/wait split, MFMA busy, L2 hits.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU -d gpurun_out/pmc_k1 -o run --output-format csv -- python3 tools/knet_bench.py > gpurun_out/pmc_k1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum -d gpurun_out/pmc_k2 -o run --output-format csv -- python3 tools/knet_bench.py > gpurun_out/pmc_k2.log 2>&1 &&
python3 - <<'PY'
import csv, glob, collections
for d in ("gpurun_out/pmc_k1", "gpurun_out/pmc_k2"):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no csv in", d); continue
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "knet_" not in k: continue
        name = k.split("::")[1].split("(")[0]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(name, r["Counter_Name"])] += 1
    for name, cs in acc.items():
        print(name, {c: round(v / n[(name, c)]) for c, v in cs.items()})
PY
