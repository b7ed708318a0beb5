"""Summarize SQ PMC passes of the fused MPC launch (the largest solve_kernel<.., true, true> dispatch):
python tools/pmc_sq.py DIR1 [DIR2 ...] -> JSON of raw counter values and derived per-instance-step ratios."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read(d):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kn = r.get("Kernel_Name", "")
            if "solve_kernel" in kn and "true, true" in kn:
                vals[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    # the timed launch: the dispatch with the most SQ_WAVE_CYCLES / GRBM_GUI_ACTIVE / first counter
    best = max(vals.values(), key=lambda v: max(v.values()))
    return dict(best)


out = {}
for d in sys.argv[1:]:
    out.update(read(d))
items = 4096 * 20
res = {"raw": out, "per_instance_step": {k: v / items for k, v in out.items()}}
if "SQ_WAVE_CYCLES" in out:
    w = out["SQ_WAVE_CYCLES"]
    res["wave_cycle_split"] = {k: out[k] / w for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS") if k in out}
if "SQ_LDS_IDX_ACTIVE" in out and "GRBM_GUI_ACTIVE" in out:
    res["lds_array_util_per_cu"] = out["SQ_LDS_IDX_ACTIVE"] / (out["GRBM_GUI_ACTIVE"] * 256)
print(json.dumps(res, indent=1))
