"""Stall breakdown of the largest fused solve_kernel dispatch from tools/pmc_stall.sh's two SQ passes.

  python tools/pmc_stall.py gpurun_out/r4s_a gpurun_out/r4s_b --out profiles/r04_pmc_stall.json

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md); the shares below are of
SQ_WAVE_CYCLES (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def largest(d):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                if ("solve_kernel" in kn or "solve_split_kernel" in kn) and "true, true" in kn:
                    per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    return max(per.values(), key=lambda c: max(c.values()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    c = {}
    for d in a.dirs:
        c.update(largest(d))
    w = c.get("SQ_WAVE_CYCLES", 0.0)
    out = {"batch": a.batch, "horizon": a.horizon, "counters": dict(c)}
    if w:
        out["share_of_wave_cycles"] = {k: c[k] / w for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                             "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                                             "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_SCA",
                                                             "SQ_INST_CYCLES_VMEM") if k in c}
    if "SQ_LDS_IDX_ACTIVE" in c and c.get("SQ_LDS_BANK_CONFLICT") is not None:
        out["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1.0)
    if "GRBM_GUI_ACTIVE" in c and "SQ_BUSY_CYCLES" in c:
        out["sq_busy_per_gui_active"] = c["SQ_BUSY_CYCLES"] / c["GRBM_GUI_ACTIVE"]
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s)
    print(s)


if __name__ == "__main__":
    main()
