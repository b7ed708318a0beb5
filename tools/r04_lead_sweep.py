"""Queue-lead sweep at the driver's command shape (B = 4096, N = 20, dt = 0.05, 5 warm-up steps then 20 timed
steps in one fused launch), two repeats per setting; prints JSON lines with the timed launch's ms."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def run(w, lead):
    L = _lib.lib()
    B, N, Ts = 4096, 20, 0.05
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    cfg = TB.config_struct(N=N, Ts=Ts)
    dev = torch.device("cuda")
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vr = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    T = 25
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev)
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev)
    hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    L.traj_debug_queue_lead(*lead)
    TB.closed_loop_run(x, u, paths, vr, cfg, None, 0, 5, hx, hu, st[:5], it[:5])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    TB.closed_loop_run(x, u, paths, vr, cfg, None, 5, 20, hx, hu, st[5:], it[5:], check=False)
    e1.record()
    torch.cuda.synchronize()
    L.traj_debug_queue_lead(1, 100)
    return e0.elapsed_time(e1)


def main():
    w = make_workload(4096, 20, 0.05, kind="spline", seed=0)
    run(w, (1, 100))
    for lead in ((1, 100), (0, 0), (2, 100), (1, 30), (1, 300), (3, 50), (1, 100)):
        ms = [run(w, lead) for _ in range(2)]
        print(json.dumps({"lead_steps": lead[0], "lead_permille": lead[1], "launch_ms": ms,
                          "rate_M": [4096 * 20 / m / 1e3 for m in ms]}), flush=True)


if __name__ == "__main__":
    main()
