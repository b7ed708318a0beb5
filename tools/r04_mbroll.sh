#!/bin/bash
# block_linearize microbenchmark variants (tools/microbench/mb_rollout_*.bin): cycles, then one SQ PMC pass each.
set -o pipefail
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${MBV:-lib fm}; do
  echo "== $v"
  timeout -k 10 60 ./tools/microbench/mb_rollout_$v.bin || exit 1
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS -d gpurun_out/mbr_$v -o run --output-format csv -- ./tools/microbench/mb_rollout_$v.bin > gpurun_out/mbr_$v.log 2>&1 || exit 1
  python3 - "$v" <<'PY'
import csv, glob, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"gpurun_out/mbr_{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
c = max(per.values(), key=lambda d: d["SQ_WAVES"])
w = c["SQ_WAVES"]
print("per instance:", {k.replace("SQ_INSTS_", ""): round(v / w, 1) for k, v in sorted(c.items()) if k != "SQ_WAVES"})
PY
done
