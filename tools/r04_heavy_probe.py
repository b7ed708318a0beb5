"""Round-4 probe: how long do the heaviest instances' 20-step chains take when they have SIMDs to themselves?

Full run (B = 4096, N = 20, dt = 0.05, bench workload): launch 1 = steps 0..4, launch 2 = steps 5..24 (timed).
Then the top-H instances of launch 2 (by ADMM iterations) re-run alone (B = H, same two launches; instances are
independent, so their histories must equal the full run's bit for bit), timed with HIP events, for 2 and 3 waves
per SIMD.  Prints JSON lines."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def run(w, idx, waves, grid=0):
    L = _lib.lib()
    L.traj_debug_fused_waves(waves)
    L.traj_debug_fused_grid(grid)
    B, N, Ts = len(idx), 20, 0.05
    paths = TB.PathSet.build(w["kinds"][idx], w["pcs"][idx], [w["knots"][i] for i in idx])
    cfg = TB.config_struct(N=N, Ts=Ts)
    dev = torch.device("cuda")
    x = torch.as_tensor(w["x0"][idx], device=dev).contiguous()
    u = torch.as_tensor(w["u0"][idx], device=dev).contiguous()
    vr = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    T = 25
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev)
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    TB.closed_loop_run(x, u, paths, vr, cfg, None, 0, 5, hx, hu, st[:5], it[:5])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    TB.closed_loop_run(x, u, paths, vr, cfg, None, 5, 20, hx, hu, st[5:], it[5:], check=False)
    e1.record()
    torch.cuda.synchronize()
    L.traj_debug_fused_waves(0)
    L.traj_debug_fused_grid(0)
    return e0.elapsed_time(e1), hx, it


def main():
    w = make_workload(4096, 20, 0.05, kind="spline", seed=0)
    allidx = np.arange(4096)
    for waves in (2, 3):
        ms, hx, it = run(w, allidx, waves)
        print(json.dumps({"what": "full", "waves": waves, "launch_ms": ms, "rate_M": 4096 * 20 / ms / 1e3}), flush=True)
    tot = it[5:].sum(0).cpu().numpy()
    order = np.argsort(-tot, kind="stable")
    print(json.dumps({"what": "iters", "top": tot[order[:64]].tolist(), "median": float(np.median(tot))}), flush=True)
    for H in (8, 32, 64):
        idx = order[:H]
        for waves in (2, 3):
            ms, hxs, _ = run(w, idx, waves)
            same = bool(torch.equal(hxs, hx[idx]))
            print(json.dumps({"what": "heavy alone", "H": H, "waves": waves, "launch_ms": ms, "same_as_full": same}),
                  flush=True)


if __name__ == "__main__":
    main()
