"""Per-launch HBM traffic of the FC2 launch (knet_fc2y_kernel by default, knet_fc2_kernel / knet_fc2x_kernel in the
other traj_knet_set_fc2_mode modes; the KalmanNet step's dominant kernel) from rocprofv3 PMC
passes (FETCH_SIZE and WRITE_SIZE in separate runs over tools/knet_bench.py):

  python tools/pmc_knet_traffic.py --fetch DIR1 --write DIR2 --batch 1024 --out profiles/traffic_knet_r01.json

Same conventions as tools/pmc_traffic.py: counters in KiB, FETCH_SIZE doubled (gfx950 correction,
MI355X_MICROARCH.md); a dispatch's value summed over its rows; only the fused runner's launches
(grid = 16 b-blocks x 32 slabs workgroups at B = 1024) are averaged."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

FC2 = re.compile(r"knet_fc2[xy]?_kernel")


def read(d, name, wgs):
    vals = defaultdict(float)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != name or not FC2.search(row.get("Kernel_Name", "")):
                    continue
                grid = int(row.get("Grid_Size", "0") or 0)
                wg = int(row.get("Workgroup_Size", "1") or 1)
                if grid // max(wg, 1) != wgs:
                    continue
                vals[row.get("Dispatch_Id")] += float(row["Counter_Value"])
    if not vals:
        raise SystemExit(f"no FC2 dispatch of {wgs} workgroups in {d}")
    return sum(vals.values()) / len(vals), len(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    wgs = ((a.batch + 63) // 64) * (10240 // 320)
    f, nf = read(a.fetch, "FETCH_SIZE", wgs)
    w, nw = read(a.write, "WRITE_SIZE", wgs)
    kib = 1024.0
    fb, wb = 2.0 * f * kib, w * kib
    # algorithmic bytes: x2 [B, 256] + W2a [10240, 256] + b2a + W2b [30, 10240] read once, partials written
    alg = 4 * (a.batch * 256 + 10240 * 256 + 10240 + 30 * 10240 + 32 * a.batch * 32)
    res = {"batch": a.batch, "dispatches": {"fetch": nf, "write": nw},
           "fetch_bytes_per_launch": {"knet_fc2": fb}, "write_bytes_per_launch": {"knet_fc2": wb},
           "hbm_bytes_per_launch": {"knet_fc2": fb + wb}, "algorithmic_bytes_per_launch": alg,
           "note": "FETCH_SIZE x2 (gfx950 correction), KiB -> bytes; the weights (12 MB) are re-read every step "
                   "from the Infinity Cache / HBM, the hidden activation never leaves the chip"}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
