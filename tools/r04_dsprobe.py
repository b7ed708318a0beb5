"""Dataset-leg probe (bench.py dataset_leg, configs[3]): B = 4096 trajectories x 240 steps from the initial
states, timed as the bench times it (run_closed_loop + pack_history, synchronized), three repeats, then the same
with the fused kernel instance forced to 2 and 3 waves per SIMD; prints JSON lines."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB, dataset as D  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main():
    B, N, Ts, T = 4096, 20, 0.05, 240
    w = make_workload(B, N, Ts, kind="spline", seed=0)
    dev = torch.device("cuda")
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=dev)
    L = _lib.lib()
    for waves in (0, 0, 2, 3):
        L.traj_debug_fused_waves(waves)
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, TB.config_struct(N=N, Ts=Ts, polish_mode=0))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            blk = D.pack_history(res["X"], res["U"], res["status"])
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            it = res["iters"].float()
            print(json.dumps({"waves": waves, "rep": rep, "run_s": t1 - t0, "pack_s": t2 - t1,
                              "rate_M": B * T / (t2 - t0) / 1e6, "iters_mean": float(it.mean()),
                              "blk": list(blk.shape)}), flush=True)
    L.traj_debug_fused_waves(0)


if __name__ == "__main__":
    main()
