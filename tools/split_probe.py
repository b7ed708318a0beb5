"""The row-split kernel (mpc_split.h) against the capacity-80 kernel (mpc_solve.h) on the same inputs, 20 < N <= 40.

  python tools/split_probe.py [N,N,...]

Per N: (1) the batch step entry point (traj_mpc_step_batch) at B = 1024 and 4096 on random parabola windows (dt 0.05)
on the capacity-80 kernel (traj_debug_split_min_n(41)) and on the row-split kernel (the default since round 6:
traj_debug_split_min_n(21)) -- time per call, statuses and u agreement; (2) config 3's closed loop (4096 mixed
references, N = 40, dt 0.05, 20 steps after 5 warmup): the fused launch on each kernel, and per-step launches on the
row-split kernel; (3) one instance at the 10,000-iteration cap re-solved alone on each (per-iteration latency).
One JSON line per measurement."""
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402
from tools.horizon_tiers import instances  # noqa: E402


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def step_compare(N, B, Ts=0.05):
    x0, up, pr, vr = instances(B, N, Ts)
    d = [torch.as_tensor(a, device="cuda") for a in (x0, up, pr, vr)]
    cfg = TB.config_struct(N=N, Ts=Ts)
    TB.set_split_min_n(41)
    dt80, o80 = timed(lambda: TB.mpc_step_batch(*d, cfg), 5)
    o80 = {k: v.cpu().numpy() for k, v in o80.items()}
    TB.set_split_min_n(21)
    dts, os_ = timed(lambda: TB.mpc_step_batch(*d, cfg), 5)
    os_ = {k: v.cpu().numpy() for k, v in os_.items()}
    TB.set_split_min_n(41)
    ok = o80["status"] <= 1
    both = ok & (o80["polished"] > 0) & (os_["polished"] > 0)
    du = np.abs(o80["u_cmd"] - os_["u_cmd"]).max(axis=1)
    print(json.dumps({"what": "step entry point", "N": N, "B": B, "cap80_ms": dt80 * 1e3, "split_ms": dts * 1e3,
                      "speedup": dt80 / dts, "status_equal": bool(np.array_equal(o80["status"], os_["status"])),
                      "iters_equal_frac": float(np.mean(o80["iters"] == os_["iters"])),
                      "du_both_polished_max": float(du[both].max(initial=0.0)),
                      "polish_agree_frac": float(np.mean((o80["polished"] > 0) == (os_["polished"] > 0)))}),
          flush=True)


def config3(N=40, B=4096, Ts=0.05, W=5, K=20, kind="mixed", tail=True):
    w = make_workload(B, N, Ts, kind=kind, seed=0)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    cfg = TB.config_struct(N=N, Ts=Ts, warm_start=1)
    res = {}
    runs = (("cap80_fused", 41, True), ("split_fused", 21, True), ("cap80_fused", 41, True), ("split_fused", 21, True))
    for name, split, fused in runs + ((("split_per_step", 21, False),) if tail else ()):
        TB.set_split_min_n(split)
        x = torch.as_tensor(w["x0"], device="cuda").clone()
        u = torch.as_tensor(w["u0"], device="cuda").clone()
        vr = torch.as_tensor(np.tile(w["vref"], (B, 1)), device="cuda").contiguous()
        T = W + K
        hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device="cuda")
        hu = torch.empty((B, T, 2), dtype=torch.float64, device="cuda")
        hx[:, 0] = x
        st = torch.empty((T, B), dtype=torch.int32, device="cuda")
        it = torch.empty((T, B), dtype=torch.int32, device="cuda")

        def run(t0, n):
            if fused:
                TB.closed_loop_run(x, u, paths, vr, cfg, None, t0, n, hx, hu, st[t0:t0 + n], it[t0:t0 + n])
            else:
                for t in range(t0, t0 + n):
                    TB.closed_loop_step(x, u, paths, vr, cfg, None, t, hx, hu, st[t], it[t])
        run(0, W)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(W, K)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        sth = st[W:].cpu().numpy().reshape(-1)
        res[name] = (hx.cpu().numpy(), hu.cpu().numpy(), it.cpu().numpy())
        print(json.dumps({"what": f"fused closed loop, {kind}, N = {N}", "path": name, "value": B * K / dt, "ms": dt * 1e3,
                          "iters_mean": float(it[W:].float().mean()),
                          "status_hist": np.bincount(sth, minlength=7).tolist()}), flush=True)
    TB.set_split_min_n(41)
    # the launch tail: one instance's steps at the 10,000-iteration cap, re-solved alone (B = 1, warm rho off: the
    # cold start reaches the cap too) on each kernel -- its per-iteration latency
    hxa, hua, ita = res["cap80_fused"]
    cap = np.argwhere(ita == 10000)
    if len(cap) and tail:
        t, bb = cap[0]
        x0 = hxa[bb, t][None]
        u0 = (hua[bb, t - 1] if t > 0 else np.asarray(w["u0"])[bb])[None]
        pr = TB.ref_window_batch(paths, x0[:, 0], np.asarray(w["vref"])[None], N, Ts).cpu().numpy()[:1]
        d = [torch.as_tensor(a_, device="cuda") for a_ in (x0, u0, pr, np.asarray(w["vref"])[None])]
        cfg0 = TB.config_struct(N=N, Ts=Ts)
        # (the one-instance slice of the path set is not needed: the step entry point takes the window)
        for name, split in (("cap80", 41), ("split", 21)):
            TB.set_split_min_n(split)
            dt, o = timed(lambda: TB.mpc_step_batch(*d, cfg0), 3)
            print(json.dumps({"what": "one capped instance alone (step entry point, B = 1)", "kernel": name,
                              "t": int(t), "b": int(bb), "ms": dt * 1e3, "iters": int(o["iters"][0]),
                              "us_per_iter": dt * 1e6 / max(int(o["iters"][0]), 1)}), flush=True)
        TB.set_split_min_n(41)


def main():
    Ns = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else "24,32,40".split(","))]
    for N in Ns:
        if N > 0:
            for B in (1024, 4096):
                step_compare(N, B)
    if "--horizons" in sys.argv:
        for N in (24, 32, 40):
            config3(N=N, kind="spline", tail=False)
    config3()


if __name__ == "__main__":
    main()
