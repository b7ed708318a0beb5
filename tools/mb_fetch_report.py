"""FETCH_SIZE per dispatch of tools/microbench/mb_fetch.hip against its known bytes.

  python tools/mb_fetch_report.py PMC_DIR MB_STDOUT.json [OUT.json]

FETCH_SIZE is rocprof's derived counter in KiB.  For each kernel: the raw counter in bytes, and its ratio to the
line bytes the kernel touches (k_run8: 21 doubles at 256-B run spacing touch 3 64-B lines = 192 B per run)."""
import csv
import glob
import json
import os
import sys

pmc, meta = sys.argv[1], json.load(open(sys.argv[2]))
vals = {}
for f in glob.glob(os.path.join(pmc, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if r.get("Counter_Name") != "FETCH_SIZE":
            continue
        for k in meta["kernels"]:
            if r["Kernel_Name"].startswith(k + "(") or r["Kernel_Name"] == k or (k + "(") in r["Kernel_Name"]:
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
res = {"what": "rocprofv3 FETCH_SIZE (KiB x 1024 = bytes) per mb_fetch.hip dispatch vs the bytes of the cache lines it "
               "touches; ratio 0.5 = the counter reports half (the guide's x2 correction applies), 1.0 = as is",
       "kernels": {}}
for k, m in meta["kernels"].items():
    f = vals.get(k)
    res["kernels"][k] = {**m, "fetch_size_bytes": f,
                         "ratio_to_line_bytes": (f / m["line_bytes"]) if f else None,
                         "ratio_to_useful_bytes": (f / m["useful_bytes"]) if f else None}
text = json.dumps(res, indent=1)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(text + "\n")
print(text)
