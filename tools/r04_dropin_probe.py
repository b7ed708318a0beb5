"""Drop-in mpc_step per-call latency (MPC/main.py's call): in-kernel linearization (default) vs the three-launch
sequence, the launch-to-sync GPU span, and a cProfile of the host side.  Prints JSON + the profile's top entries."""
import cProfile
import json
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import mpc_6stati as M  # noqa: E402
sys.path.insert(0, "tools")
from r04_tiers import instances  # noqa: E402


def per_call(x0, up, pr, vr, N, Ts, n=200):
    lat = []
    for i in range(n):
        t0 = time.perf_counter()
        M.mpc_step(x0[i % len(x0)], up[i % len(x0)], pr[i % len(x0)], Ts=Ts, N=N, vref=vr[i % len(x0)])
        lat.append(time.perf_counter() - t0)
    return 1e6 * float(np.median(lat[10:]))


def main():
    N, Ts = 20, 0.05
    x0, up, pr, vr = instances(64, N, Ts)
    L = _lib.lib()
    for mode in (1, 0):
        L.traj_debug_step_linearize(mode)
        per_call(x0, up, pr, vr, N, Ts, 20)
        us = per_call(x0, up, pr, vr, N, Ts)
        print(json.dumps({"N": N, "step_linearize_in_kernel": mode, "dropin_call_us_median": us}), flush=True)
    L.traj_debug_step_linearize(1)
    # GPU span of one call's launch (events around the batch call at B = 1)
    from trajectory_generation_amd import batch as TB
    cfg = TB.config_struct(N=N, Ts=Ts)
    d = [torch.as_tensor(a[:1], device="cuda") for a in (x0, up, pr, vr)]
    for mode in (1, 0):
        L.traj_debug_step_linearize(mode)
        TB.mpc_step_batch(*d, cfg)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(50):
            e0.record(); TB.mpc_step_batch(*d, cfg); e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"B": 1, "step_linearize_in_kernel": mode, "gpu_span_us_median": float(np.median(ts))}), flush=True)
    L.traj_debug_step_linearize(1)
    pr_ = cProfile.Profile()
    pr_.enable()
    per_call(x0, up, pr, vr, N, Ts, 200)
    pr_.disable()
    st = pstats.Stats(pr_)
    st.sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
