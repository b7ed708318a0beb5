"""traj_mpc_step_batch throughput at B = 1024 / 4096 (N = 20, dt = 0.05): linearization inside the solve launch
(default) vs the rollout + Jacobian + solve launches.  Prints JSON lines."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from r04_tiers import instances  # noqa: E402


def main():
    N, Ts = 20, 0.05
    L = _lib.lib()
    for B in (1024, 4096):
        d = [torch.as_tensor(a, device="cuda") for a in instances(B, N, Ts)]
        cfg = TB.config_struct(N=N, Ts=Ts)
        for mode in (1, 0, 1, 0):
            L.traj_debug_step_linearize(mode)
            TB.mpc_step_batch(*d, cfg)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                TB.mpc_step_batch(*d, cfg)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / 5
            print(json.dumps({"B": B, "in_kernel": mode, "ms": dt * 1e3, "steps_per_s": B / dt}), flush=True)
    L.traj_debug_step_linearize(1)


if __name__ == "__main__":
    main()
