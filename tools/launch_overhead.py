"""Host-side cost of one fused closed-loop launch at the bench workload (4096 trajectories, N = 20,
dt = 0.05, 20 steps): wall time of the traj_closed_loop_run call itself, of the hand-off check, and of
the whole run to synchronize, with and without the bench's per-kernel event timing armed.

  python tools/launch_overhead.py > gpurun_out/launch_overhead.json
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main():
    B, N, Ts, K = 4096, 20, 0.05, 20
    dev = torch.device("cuda:0")
    w = make_workload(B, N, Ts, kind="spline", seed=0)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=dev)
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    T = 5 + 6 * K
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev)
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    TB.closed_loop_run(x, u, paths, vref, cfg, None, 0, 5, hx, hu, st[:5], it[:5])
    torch.cuda.synchronize()
    L = _lib.lib()
    out = []
    t0s = 5
    for rep in range(6):
        timing = rep % 2 == 1
        if timing:
            _lib.check(L.traj_debug_kernel_timing(K), "timing")
        torch.cuda.synchronize()
        a = time.perf_counter()
        TB.closed_loop_run(x, u, paths, vref, cfg, None, t0s, K, hx, hu, st[t0s:t0s + K], it[t0s:t0s + K], check=False)
        b = time.perf_counter()
        _lib.check(L.traj_closed_loop_check(TB._p(TB.workspace(B, N, dev)), TB.workspace(B, N, dev).numel() * 8, B, N,
                                            TB._stream()), "check")
        c = time.perf_counter()
        torch.cuda.synchronize()
        d = time.perf_counter()
        rec = {"timing_armed": timing, "launch_call_ms": 1e3 * (b - a), "check_ms": 1e3 * (c - b),
               "total_ms": 1e3 * (d - a)}
        if timing:
            ms = (ctypes.c_double * 4)()
            n = ctypes.c_int(0)
            L.traj_debug_kernel_times(ms, ctypes.byref(n))
            rec["event_ms"] = {"memset..stamp2": ms[0] + ms[1], "order_kernel": ms[2], "solve_kernel": ms[3]}
            _lib.check(L.traj_debug_kernel_timing(0), "timing off")
        out.append(rec)
        t0s += K
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
