"""Issue-side view of the fused MPC launch from one SQ PMC pass (tools/pmc_f64.sh).

  python tools/pmc_f64.py DIR --batch 4096 --steps-per-launch 20 --out profiles/sq_f64_r01.json

Counters are wave-instruction counts summed over the launch; the largest fused solve_kernel dispatch
(the timed K-step launch) is kept.  f64 lane-FLOP issued = 64 x (ADD + MUL + TRANS + 2 FMA) + 512 x
MFMA_MOPS_F64 (one MOPS unit = 512 FLOP).  Masked lanes count as issued: the solve runs 40 QP rows
on 64 lanes, so this is what the SIMDs were asked to do, an upper bound on useful FLOP.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

NAMES = ("SQ_INSTS_VALU", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
         "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_WAVES")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--steps-per-launch", type=int, required=True)
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {a.dir}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                kn = row.get("Kernel_Name", "")
                if ("solve_kernel" in kn or "solve_split_kernel" in kn) and "true, true" in kn and row.get("Counter_Name") in NAMES:
                    per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        raise SystemExit("no fused solve_kernel dispatch")
    c = max(per.values(), key=lambda d: d.get("SQ_INSTS_VALU", 0.0))
    units = a.batch * a.steps_per_launch
    f64_valu = 64.0 * (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_TRANS_F64"]
                       + 2.0 * c["SQ_INSTS_VALU_FMA_F64"])
    f64_mfma = 512.0 * c["SQ_INSTS_VALU_MFMA_MOPS_F64"]
    out = {"batch": a.batch, "horizon": a.horizon, "steps_per_launch": a.steps_per_launch, "counters_per_launch": dict(c),
           "valu_insts_per_step": c["SQ_INSTS_VALU"] / units,
           "f64_valu_insts_per_step": (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"]
                                       + c["SQ_INSTS_VALU_TRANS_F64"] + c["SQ_INSTS_VALU_FMA_F64"]) / units,
           "f64_flop_issued_per_step": (f64_valu + f64_mfma) / units,
           "f64_mfma_flop_per_step": f64_mfma / units,
           "note": "wave-instruction counts of the largest fused solve_kernel dispatch; FLOP = 64 lanes x "
                   "(ADD+MUL+TRANS+2 FMA) + 512 x MFMA_MOPS_F64, masked lanes included"}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
