"""Queue-lead / grid sweep of the fused closed loop at the bench's workload (B=4096 spline trajectories, N=20,
dt=0.05): for every (lead_steps, lead_permille, grid) given, the bench's sequence -- a 5-step warmup launch, then
one timed launch of K steps -- from the same initial states, and the MPC steps/s of the timed launch.

  python tools/r03_sweep.py --steps 20 200 --lead 1:100 2:50 --grid 0
(TRAJMPC_LIB selects a library build; grid 0 = the resident slots.)
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def run(w, dev, B, N, Ts, warm, steps):
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=dev)
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    T = warm + steps
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev)
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    TB.closed_loop_run(x, u, paths, vref, cfg, None, 0, warm, hx, hu, st[:warm], it[:warm])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    TB.closed_loop_run(x, u, paths, vref, cfg, None, warm, steps, hx, hu, st[warm:], it[warm:])
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return B * steps / dt, it[warm:].cpu().numpy(), hx, hu


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, nargs="+", default=[20, 200])
    ap.add_argument("--lead", nargs="+", default=["1:100"], help="lead_steps:lead_permille")
    ap.add_argument("--grid", type=int, nargs="+", default=[0])
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    dev = TB.require_gpu("cuda:0")
    B, N, Ts = 4096, 20, 0.05
    w = make_workload(B, N, Ts, kind="spline", seed=0, id_offset=0)
    L = _lib.lib()
    if hasattr(L, "traj_debug_fused_waves") and os.environ.get("FUSED_WAVES"):
        _lib.check(L.traj_debug_fused_waves(int(os.environ["FUSED_WAVES"])), "waves")
    ref = {}
    for g in args.grid:
        _lib.check(L.traj_debug_fused_grid(g), "grid")
        for ld in args.lead:
            s, pm = (int(v) for v in ld.split(":"))
            _lib.check(L.traj_debug_queue_lead(s, pm), "lead")
            for K in args.steps:
                vals = []
                for _ in range(args.reps):
                    v, its, hx, hu = run(w, dev, B, N, Ts, 5, K)
                    vals.append(v)
                # bit-identity across configurations (the queue order never changes a result; NaN == NaN)
                same = None
                eq = lambda a, b: bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())  # noqa: E731
                if K in ref:
                    same = eq(ref[K][0], hx) and eq(ref[K][1], hu)
                else:
                    ref[K] = (hx, hu)
                print(json.dumps({"grid": g, "lead": ld, "steps": K, "value": max(vals), "values": vals,
                                  "iters_mean": float(its.mean()), "bit_identical": same}), flush=True)
    _lib.check(L.traj_debug_fused_grid(0), "grid")


if __name__ == "__main__":
    main()
