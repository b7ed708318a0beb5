"""Determinism check of the fused closed loop at the bench workload: the same 5 + K-step sequence run several
times (same queue lead, then other leads); for every pair of runs that differ, the first differing
(trajectory, step), its status / iteration history in both runs, and how many trajectories differ."""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from r03_sweep import run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--lead", nargs="+", default=["1:100", "1:100", "2:100", "0:0"])
    ap.add_argument("--batch", type=int, default=4096)
    args = ap.parse_args()
    dev = TB.require_gpu("cuda:0")
    B, N, Ts = args.batch, 20, 0.05
    w = make_workload(B, N, Ts, kind="spline", seed=0, id_offset=0)
    L = _lib.lib()
    runs = []
    for ld in args.lead:
        s, pm = (int(v) for v in ld.split(":"))
        _lib.check(L.traj_debug_queue_lead(s, pm), "lead")
        v, its, hx, hu = run(w, dev, B, N, Ts, 5, args.steps)
        runs.append((ld, hx.cpu().numpy(), hu.cpu().numpy(), its))
    _lib.check(L.traj_debug_queue_lead(1, 100), "lead")
    ld0, X0, U0, I0 = runs[0]
    for ld, X, U, I in runs[1:]:
        dx = ~((X == X0) | (np.isnan(X) & np.isnan(X0))).all(axis=2)      # [B, T+1]
        bad = np.where(dx.any(axis=1))[0]
        rec = {"ref": ld0, "run": ld, "n_traj_differ": int(bad.size)}
        if bad.size:
            firsts = [(int(b), int(np.argmax(dx[b]))) for b in bad]
            firsts.sort(key=lambda x: x[1])
            rec["first"] = firsts[:10]
            b, t = firsts[0]
            rec["b"] = b
            rec["x_ref"] = X0[b, max(t - 1, 0):t + 1].tolist()
            rec["x_run"] = X[b, max(t - 1, 0):t + 1].tolist()
            rec["iters_ref"] = I0[max(t - 6, 0):t + 1, b].tolist() if t - 6 < I0.shape[0] else None
            rec["iters_run"] = I[max(t - 6, 0):t + 1, b].tolist() if t - 6 < I.shape[0] else None
            rec["max_abs_x_ref"] = float(np.nanmax(np.abs(X0[b])))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
