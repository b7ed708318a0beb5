"""Per-phase cycles of the row-split kernel's fused closed loop (mpc_split.h DIAG stamps; diagnostics only).

  python tools/split_phase.py [N] [kind] [steps] [B]   (defaults: 40 mixed 20 4096 -- config 3)

Runs W = 5 fused steps, then one stamped fused launch of `steps` steps (the stamped instance: solve_split_kernel with
DIAG = true), and prints per-phase cycle statistics of each instance's last step from s_memtime stamps (one workgroup,
one XCD per item): inputs + window, linearization, condensing, Ruiz / scaling, the sweeps (all factorizations), the
ADMM iterations, the polish, the outputs / plant update, and per-iteration ADMM cycles.  Items that end before the ADMM
(solver error, infeasible up front) or whose stamps are not monotone are counted and left out."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main(N=40, kind="mixed", steps=20, B=4096, Ts=0.05, W=5):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind=kind, seed=0)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    cfg = TB.config_struct(N=N, Ts=Ts, warm_start=1)
    x = torch.as_tensor(w["x0"], device=dev).clone()
    u = torch.as_tensor(w["u0"], device=dev).clone()
    vr = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    TB.closed_loop_run(x, u, paths, vr, cfg, None, 0, W)
    torch.cuda.synchronize()
    dbg = torch.zeros((B, 32), dtype=torch.int64, device=dev)
    _lib.lib().traj_debug_set_stamps(C.c_void_p(dbg.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    try:
        e0.record()
        TB.closed_loop_run(x, u, paths, vr, cfg, None, W, steps)
        e1.record()
        torch.cuda.synchronize()
    finally:
        _lib.lib().traj_debug_set_stamps(None)
    d = dbg.cpu().numpy().astype(np.float64)
    seq = d[:, [0, 1, 2, 3, 4, 6, 7]]
    ok = (np.diff(seq, axis=1) >= 0).all(axis=1) & (d[:, 9] > 0) & (d[:, 0] > 0)
    ok &= (seq[:, -1] - seq[:, 0]) < 5e9
    d = d[ok]
    sweep_per = d[:, 5] / np.maximum(d[:, 8], 1)
    ph = {
        "inputs+window": d[:, 1] - d[:, 0],
        "linearization": d[:, 2] - d[:, 1],
        "condensing": d[:, 3] - d[:, 2],
        "  condensing: sensitivities (wave 0)": d[:, 12],
        "  condensing: products (wave 0)": d[:, 13],
        "  condensing: barrier waits (wave 0)": d[:, 14],
        "scaling": d[:, 4] - d[:, 3],
        "solve (ADMM + sweeps + polish)": d[:, 6] - d[:, 4],
        "sweeps (every factorization)": d[:, 5],
        "  sweeps: pivot barrier waits (wave 0)": d[:, 15],
        "  sweeps: barrier -> reciprocal and pivot-row branch done (wave 0)": d[:, 17],
        "  sweeps: the row update (wave 0)": d[:, 18],
        "polish pass (its sweep included)": d[:, 10],
        "admm iterations": (d[:, 6] - d[:, 4]) - d[:, 10] - sweep_per * (d[:, 8] - (d[:, 10] > 0)),
        "outputs+plant": d[:, 7] - d[:, 6],
        "barrier waits in exchanges / broadcasts (wave 0, whole item)": d[:, 16],
        "total": d[:, 7] - d[:, 0],
    }
    it = d[:, 9]
    res = {"N": N, "kind": kind, "B": B, "steps": steps, "launch_ms": e0.elapsed_time(e1),
           "items": int(ok.sum()), "left_out": int((~ok).sum()),
           "iters": {"median": float(np.median(it)), "mean": float(it.mean()), "max": float(it.max())},
           "factorizations_median": float(np.median(d[:, 8])),
           "phases_cycles": {k: {"median": float(np.median(v)), "mean": float(v.mean()), "p90": float(np.percentile(v, 90))}
                             for k, v in ph.items()}}
    res["admm_cycles_per_iter_median"] = float(np.median(ph["admm iterations"] / np.maximum(it, 1)))
    res["sweep_cycles_per_factorization_median"] = float(np.median(sweep_per))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(N=int(a[0]) if len(a) > 0 else 40, kind=a[1] if len(a) > 1 else "mixed", steps=int(a[2]) if len(a) > 2 else 20,
         B=int(a[3]) if len(a) > 3 else 4096)
