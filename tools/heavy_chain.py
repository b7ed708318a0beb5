"""Where the critical chain's time goes: per-step solve counters of the heaviest instances (diagnostics only).

  python tools/heavy_chain.py [steps] [warmup] [top]

The driver's workload (4096 spline trajectories, N = 20, dt = 0.05): `warmup` per-step launches, then `steps`
per-step launches with traj_debug_set_stamps, and for the `top` instances with the most ADMM iterations over those
steps, per step: iterations, factorizations (ADMM + rho changes + polish), residual checks, and the cycles of the
sweeps, residual checks, polish and the whole item (wall cycles in a launch shared with the other instances).
The per-step launches are bit-identical to the fused run (test_fused_closed_loop_bit_identical)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main(steps=20, warm=5, top=8, B=4096, N=20, Ts=0.05):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind="spline")
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    for t in range(warm):
        TB.closed_loop_step(x, u, paths, vref, cfg, None, t)
    dbg = torch.zeros((B, 32), dtype=torch.int64, device=dev)
    rec = []
    for s in range(steps):
        dbg.zero_()
        _lib.lib().traj_debug_set_stamps(C.c_void_p(dbg.data_ptr()))
        TB.closed_loop_step(x, u, paths, vref, cfg, None, warm + s)
        torch.cuda.synchronize()
        _lib.lib().traj_debug_set_stamps(None)
        d = dbg.cpu().numpy()
        rec.append({"iters": d[:, 9].copy(), "nfact": d[:, 8].copy(), "n_res": d[:, 14].copy(),
                    "cyc_res": d[:, 11].copy(), "cyc_sweep": d[:, 12].copy(), "cyc_pol": d[:, 13].copy(),
                    "total": (d[:, 7] - d[:, 0]).copy()})
    it = np.stack([r["iters"] for r in rec])          # [steps, B]
    order = np.argsort(-it.sum(0))[:top]
    out = {"steps": steps, "warmup": warm, "B": B, "N": N, "instances": []}
    for b in order:
        per = [{k: int(r[k][b]) for k in rec[0]} for r in rec]
        tot = {k: int(sum(p[k] for p in per)) for k in per[0]}
        out["instances"].append({"b": int(b), "sum": tot, "per_step": per})
    allv = {k: float(np.mean([r[k].mean() for r in rec])) for k in rec[0]}
    out["mean_over_instances_per_step"] = allv
    print(json.dumps(out))


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:4]]
    main(*a)
