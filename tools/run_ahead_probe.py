"""Fused closed loop with and without run-ahead (traj_debug_run_ahead; diagnostics only).

  python tools/run_ahead_probe.py [levels ...]

For each workload (the bench's N = 20 spline line and config 3's N = 40 mixed line, 4096 trajectories, 5 warmup
steps then one 20-step fused launch, as bench.py) and each run-ahead setting: the timed launch by HIP events
(best of 3 fresh runs) and whether the histories equal the run-ahead-0 run's bit for bit.  RA_N=20|40 runs one
workload; RA_SEED=s another workload seed; RA_OUT=path writes the JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def once(w, B, N, Ts, warm, steps, dev):
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=dev)
    cfg = TB.config_struct(N=N, Ts=Ts)
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    T = warm + steps
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev)
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    if warm:
        TB.closed_loop_run(x, u, paths, vref, cfg, None, 0, warm, hx, hu, st[:warm], it[:warm])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    TB.closed_loop_run(x, u, paths, vref, cfg, None, warm, steps, hx, hu, st[warm:], it[warm:])
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1), (hx.cpu(), hu.cpu(), st.cpu(), it.cpu())


def main(levels):
    dev = TB.require_gpu()
    L = _lib.lib()
    B, Ts = 4096, 0.05
    warm, steps = int(os.environ.get("RA_WARM", 5)), int(os.environ.get("RA_STEPS", 20))   # (240, 0: configs[3])
    out = {}
    cases = ((20, "spline"), (40, "mixed"))
    if os.environ.get("RA_N"):   # one horizon only (20: spline, 40: mixed)
        cases = tuple(c for c in cases if c[0] == int(os.environ["RA_N"]))
    seed = int(os.environ["RA_SEED"]) if os.environ.get("RA_SEED") else None   # None: the bench's workload
    for N, kind in cases:
        w = make_workload(B, N, Ts, kind=kind) if seed is None else make_workload(B, N, Ts, kind=kind, seed=seed)
        ref = None
        for R in [0] + [r for r in levels if r != 0]:
            _lib.check(L.traj_debug_run_ahead(R), "traj_debug_run_ahead")
            ms, hist = [], None
            for _ in range(3):
                m, h = once(w, B, N, Ts, warm, steps, dev)
                ms.append(m)
                hist = h
            if ref is None:
                ref = hist
            same = all(bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all()) for a, b in zip(hist, ref))
            best = min(ms)
            r = {"ms": [round(v, 3) for v in ms], "best_ms": round(best, 3),
                 "steps_per_s_M": round(B * steps / best / 1e3, 3), "bit_identical_to_R0": same}
            out[f"N{N}_R{R}"] = r
            print(f"N={N} {kind} run_ahead={R}: {r}", flush=True)
    _lib.check(L.traj_debug_run_ahead(0), "traj_debug_run_ahead")
    path = os.environ.get("RA_OUT")
    if path:
        with open(path, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main([int(v) for v in sys.argv[1:]] or [2, 4, 8])
