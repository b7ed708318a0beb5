"""Per-step solve_kernel time vs the step's iteration statistics (diagnostics only): is the solve
launch bound by the total work of the batch or by its slowest instance?"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main(B=4096, N=20, Ts=0.05, steps=205, kind="spline"):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind=kind)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    L = _lib.lib()
    st = torch.empty((steps, B), dtype=torch.int32, device=dev)
    it = torch.empty((steps, B), dtype=torch.int32, device=dev)
    ms = np.zeros((steps, 4))
    buf, n = (C.c_double * 4)(), C.c_int()
    for t in range(steps):
        L.traj_debug_kernel_timing(1)
        TB.closed_loop_step(x, u, paths, vref, cfg, None, t, None, None, st[t], it[t])
        L.traj_debug_kernel_times(buf, C.byref(n))
        ms[t] = list(buf)
    L.traj_debug_kernel_timing(0)
    I = it.cpu().numpy()
    s = ms[5:, 3]
    mx, sm = I[5:].max(1), I[5:].sum(1)
    print(f"solve ms: mean {s.mean():.3f} min {s.min():.3f} max {s.max():.3f}")
    print(f"iters per step: mean-of-mean {I[5:].mean():.1f}, max per step: median {np.median(mx):.0f} max {mx.max()}")
    A = np.stack([sm / B, mx, np.ones_like(mx)], 1).astype(float)
    coef, *_ = np.linalg.lstsq(A, s, rcond=None)
    pred = A @ coef
    r2 = 1 - ((s - pred) ** 2).sum() / ((s - s.mean()) ** 2).sum()
    print("solve_ms ~ %.4f * mean_iters + %.5f * max_iters + %.3f   (R^2 %.3f)" % (*coef, r2))
    print("corr(solve, mean iters) %.3f  corr(solve, max iters) %.3f" % (np.corrcoef(s, sm)[0, 1], np.corrcoef(s, mx)[0, 1]))
    order = np.argsort(s)
    for k in list(order[:3]) + list(order[-5:]):
        print(f"  step {k + 5:3d}: solve {s[k]:.3f} ms, mean iters {sm[k] / B:.1f}, max iters {mx[k]}, "
              f">=500: {(I[k + 5] >= 500).sum()}")


if __name__ == "__main__":
    main()
