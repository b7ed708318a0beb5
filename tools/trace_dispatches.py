"""Per-dispatch durations of one kernel from a rocprofv3 --kernel-trace CSV (the stats file averages the
warmup launch with the timed one): python tools/trace_dispatches.py TRACE.csv KERNEL_SUBSTRING [OUT.json]"""
import csv
import json
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        rows.append({"dispatch": int(r["Dispatch_Id"]), "grid_x": int(r["Grid_Size_X"]),
                     "workgroup_x": int(r["Workgroup_Size_X"]), "vgpr": int(r["VGPR_Count"]),
                     "agpr": int(r["Accum_VGPR_Count"]), "scratch": int(r["Scratch_Size"]),
                     "lds": int(r["LDS_Block_Size"]),
                     "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
out = {"trace": sys.argv[1], "kernel": sys.argv[2], "dispatches": rows}
text = json.dumps(out, indent=1)
if len(sys.argv) > 3:
    open(sys.argv[3], "w").write(text + "\n")
print(text)
