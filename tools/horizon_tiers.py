"""Horizon tiers (include/trajmpc.h): per-step batch throughput of traj_mpc_step_batch at B = 1024
(random parabola windows, dt = 0.05) for horizons in each kernel tier (one wave N <= 20, two waves 20 < N <= 40, the
long-horizon kernel 40 < N <= 128), and the drop-in mpc_step per-call time (median of 20).  One JSON line per N.
  python tools/horizon_tiers.py [N,N,...]"""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd import mpc_6stati as M  # noqa: E402


def instances(B, N, Ts, seed=0):
    rng = np.random.default_rng(seed)
    v = TB.vref_ramp(N, Ts)
    x0 = np.stack([rng.uniform(-2, 2, B), rng.uniform(-2, 2, B), rng.uniform(-0.3, 0.3, B), rng.uniform(0.4, 1.5, B),
                   rng.uniform(-.05, .05, B), rng.uniform(-1, 1, B)], 1)
    up = np.stack([rng.uniform(-0.2, 0.5, B), rng.uniform(-0.3, 0.3, B)], 1)
    pr = np.zeros((B, N + 1, 3))
    for b in range(B):
        xs = x0[b, 0] + np.concatenate([[0], np.cumsum(v[:-1] * Ts)])
        pr[b] = np.stack([xs, 0.1 * xs ** 2, np.arctan(0.2 * xs)], 1)
    return x0, up, pr, np.tile(v, (B, 1))


def main():
    Ts, B = 0.05, 1024
    for N in [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "8,20,24,30,32,40,41,60,64,65,100,128".split(","))]:
        x0, up, pr, vr = instances(B, N, Ts)
        d = [torch.as_tensor(a, device="cuda") for a in (x0, up, pr, vr)]
        cfg = TB.config_struct(N=N, Ts=Ts)
        TB.mpc_step_batch(*d, cfg)
        torch.cuda.synchronize()
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            o = TB.mpc_step_batch(*d, cfg)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        st = o["status"].cpu().numpy()
        # drop-in per call (the reference's mpc_step signature), median of 20 calls
        calls = []
        for i in range(21):
            t1 = time.perf_counter()
            M.mpc_step(x0[i], up[i], pr[i], Ts=Ts, N=N, vref=vr[i])
            calls.append(time.perf_counter() - t1)
        print(json.dumps({"N": N, "B": B, "batch_ms": dt * 1e3, "steps_per_s": B / dt,
                          "optimal_frac": float((st <= 1).mean()), "dropin_call_us_median": 1e6 * float(np.median(calls[1:]))}),
              flush=True)


if __name__ == "__main__":
    main()
