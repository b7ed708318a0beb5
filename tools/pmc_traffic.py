"""Per-launch HBM traffic of the MPC step from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE
collected in separate runs, MI355X_MICROARCH.md "rocprofv3 PMC slots").

  python tools/pmc_traffic.py --fetch DIR1 --write DIR2 --batch 4096 --horizon 20 --out profiles/traffic_r01.json

FETCH_SIZE / WRITE_SIZE are rocprof derived counters in KiB.  gfx950 correction (same guide, "HBM"):
FETCH_SIZE counts 128-B requests at 64 B, so it is doubled; WRITE_SIZE is taken as is.  Only the
bench's own launches are kept (grid = batch workgroups).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = ("rollout_kernel", "jac_kernel", "order_kernel", "solve_kernel")


def expected_blocks(batch, horizon):
    """Workgroups of each bench launch (trajmpc.hip traj_closed_loop_step)."""
    return {"rollout_kernel": (batch + 63) // 64, "jac_kernel": (batch * horizon + 63) // 64, "order_kernel": 1,
            "solve_kernel": batch}


def read_counter_fused(d, name):
    """Fused closed loop: the largest solve_kernel<.., true, true> dispatch (the timed K-step launch)."""
    vals = defaultdict(float)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == name and ("solve_kernel" in row.get("Kernel_Name", "")
                                                        or "solve_split_kernel" in row.get("Kernel_Name", "")) \
                        and "true, true" in row.get("Kernel_Name", ""):
                    vals[row.get("Dispatch_Id")] += float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no fused solve_kernel dispatch in {d}")
    return max(vals.values())


def read_counter(d, name, batch, horizon):
    want = expected_blocks(batch, horizon)
    vals = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != name:
                    continue
                kn = row.get("Kernel_Name", "")
                k = next((k for k in KERNELS if k in kn), None)
                if k is None:
                    continue
                grid = int(row.get("Grid_Size", "0") or 0)
                wg = int(row.get("Workgroup_Size", "1") or 1)
                if grid // max(wg, 1) != want[k]:
                    continue
                vals[(k, row.get("Dispatch_Id"))].append(float(row["Counter_Value"]))
    per_kernel = defaultdict(list)
    for (k, _), v in vals.items():
        per_kernel[k].append(sum(v))   # a dispatch's value may be split over several rows (per XCD/SE)
    return {k: sum(v) / len(v) for k, v in per_kernel.items()}, {k: len(v) for k, v in per_kernel.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--out", required=True)
    ap.add_argument("--fused-steps", type=int, default=0,
                    help="fused closed loop (bench default): K steps per launch; report that launch")
    a = ap.parse_args()
    if a.fused_steps:
        kib = 1024.0
        fb = 2.0 * read_counter_fused(a.fetch, "FETCH_SIZE") * kib
        wb = read_counter_fused(a.write, "WRITE_SIZE") * kib
        res = {"batch": a.batch, "horizon": a.horizon, "fused": True, "steps_per_launch": a.fused_steps,
               "fetch_bytes_per_launch": {"solve_kernel": fb}, "write_bytes_per_launch": {"solve_kernel": wb},
               "hbm_bytes_per_kernel": {"solve_kernel": fb + wb}, "hbm_bytes_per_launch": fb + wb,
               "hbm_bytes_per_step": (fb + wb) / a.fused_steps,
               "hbm_bytes_per_instance_step": (fb + wb) / (a.fused_steps * a.batch),
               "note": "fused traj_closed_loop_run launch of fused_steps steps; FETCH_SIZE x2 (gfx950 correction), "
                       "KiB -> bytes"}
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res, indent=1))
        return
    fetch, nf = read_counter(a.fetch, "FETCH_SIZE", a.batch, a.horizon)
    write, nw = read_counter(a.write, "WRITE_SIZE", a.batch, a.horizon)
    kib = 1024.0
    res = {"batch": a.batch, "horizon": a.horizon, "dispatches": {"fetch": nf, "write": nw},
           "raw_kib": {"FETCH_SIZE": fetch, "WRITE_SIZE": write},
           "fetch_bytes_per_launch": {k: 2.0 * v * kib for k, v in fetch.items()},
           "write_bytes_per_launch": {k: v * kib for k, v in write.items()}}
    res["hbm_bytes_per_kernel"] = {k: res["fetch_bytes_per_launch"].get(k, 0.0) + res["write_bytes_per_launch"].get(k, 0.0)
                                   for k in KERNELS}
    res["hbm_bytes_per_launch"] = sum(res["hbm_bytes_per_kernel"].values())
    res["note"] = ("hbm_bytes_per_launch = one closed-loop step (rollout + jac + order + solve launches); "
                   "FETCH_SIZE x2 (gfx950 correction), KiB -> bytes")
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
