"""Latency of one MPC step at B = 1 (the drop-in call; diagnostics only).

  python tools/dropin_probe.py [calls]

(a) the drop-in mpc_6stati.mpc_step per call (host staging, one launch, one copy back, synchronize), median;
(b) the launch alone by HIP events (batch.mpc_step_batch on device tensors), back to back and with a 2 ms host
    pause before each call (the closed loop's host work between calls);
(c) the kernel's own cycles and clock (traj_debug_set_stamps: s_memtime / s_memrealtime) in both regimes."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB, mpc_6stati as M  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main(calls=200, N=20, Ts=0.05):
    dev = TB.require_gpu()
    w = make_workload(8, N, Ts, kind="spline", seed=4)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    vr = np.tile(w["vref"], (1, 1))
    x0 = np.asarray(w["x0"][:1]); u0 = np.asarray(w["u0"][:1])
    pr = TB.ref_window_batch(paths, x0[:, 0], np.tile(w["vref"], (8, 1))[:1], N, Ts).cpu().numpy()
    res = {"N": N, "Ts": Ts}
    # (a) the drop-in call
    for _ in range(10):
        M.mpc_step(x0[0], u0[0], pr[0], Ts=Ts, N=N, vref=vr[0])
    t = []
    for _ in range(calls):
        t0 = time.perf_counter()
        M.mpc_step(x0[0], u0[0], pr[0], Ts=Ts, N=N, vref=vr[0])
        t.append(time.perf_counter() - t0)
    if os.environ.get("DP_PROF"):   # where the host part of the call goes
        import cProfile
        import pstats
        pr_ = cProfile.Profile()
        pr_.enable()
        for _ in range(calls):
            M.mpc_step(x0[0], u0[0], pr[0], Ts=Ts, N=N, vref=vr[0])
        pr_.disable()
        pstats.Stats(pr_).sort_stats("tottime").print_stats(25)
    res["dropin_call_us_median"] = 1e6 * float(np.median(t))
    res["dropin_call_us_p10"] = 1e6 * float(np.percentile(t, 10))
    # (b, c) the launch alone, on device tensors
    cfg = TB.config_struct(N=N, Ts=Ts)
    xd, ud = torch.as_tensor(x0, device=dev), torch.as_tensor(u0, device=dev)
    prd, vrd = torch.as_tensor(pr, device=dev), torch.as_tensor(vr, device=dev)
    out = TB.mpc_step_batch(xd, ud, prd, vrd, cfg)
    dbg = torch.zeros((1, 32), dtype=torch.int64, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for mode, pause in (("back_to_back", 0.0), ("after_2ms_pause", 2e-3)):
        ms, cyc, clk = [], [], []
        for i in range(calls):
            if pause:
                time.sleep(pause)
            stamp = (i % 4 == 0)
            if stamp:
                _lib.lib().traj_debug_set_stamps(C.c_void_p(dbg.data_ptr()))
            e0.record()
            TB.mpc_step_batch(xd, ud, prd, vrd, cfg, out=out)
            e1.record()
            e1.synchronize()
            if stamp:
                _lib.lib().traj_debug_set_stamps(None)
                d = dbg.cpu().numpy()[0]
                tot, wall = float(d[7] - d[0]), float(d[3] - d[2])   # s_memtime cycles; 100 MHz ticks
                if tot > 0 and wall > 0:
                    cyc.append(tot)
                    clk.append(0.1 * tot / wall)
                    last = d.copy()
            else:
                ms.append(e0.elapsed_time(e1))
        res[mode] = {"launch_us_median": 1e3 * float(np.median(ms)), "kernel_cycles_median": float(np.median(cyc)),
                     "clock_GHz_median": float(np.median(clk)), "stamped_calls": len(cyc)}
        # the last stamped call's phases (cycles): slots as tools/phase_profile.py (20 / 21: in-kernel linearization)
        res[mode]["phases_last_call"] = {
            "inputs+linearization": int(last[1] - last[0]), "condense": int(last[4] - last[1]),
            "scale": int(last[5] - last[4]), "solve": int(last[6] - last[5]), "outputs": int(last[7] - last[6]),
            "stage_loop": int(last[18] - last[17]), "sweeps": int(last[12]), "polish": int(last[13]),
            "residual_checks": int(last[11]), "iters": int(last[9]), "factorizations": int(last[8]),
            "stamps_0_1_20_21_16": [int(last[i] - last[0]) for i in (0, 1, 20, 21, 16)]}
    print(json.dumps(res))
    if os.environ.get("DP_OUT"):
        with open(os.environ["DP_OUT"], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
