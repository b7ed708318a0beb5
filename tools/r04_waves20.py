"""Waves per SIMD x queue lead at the driver's command shape (B = 4096, N = 20, dt = 0.05, 5 warm-up steps then 20
timed steps in one fused launch), two repeats per setting; prints JSON lines with the timed launch's ms."""
import json
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402
from r04_lead_sweep import run  # noqa: E402


def main():
    L = _lib.lib()
    w = make_workload(4096, 20, 0.05, kind="spline", seed=0)
    run(w, (1, 100))
    for waves in (2, 3):
        L.traj_debug_fused_waves(waves)
        for lead in ((1, 100), (1, 300), (2, 300), (4, 300), (2, 500)):
            ms = [run(w, lead) for _ in range(2)]
            print(json.dumps({"waves": waves, "lead_steps": lead[0], "lead_permille": lead[1], "launch_ms": ms,
                              "rate_M": [4096 * 20 / m / 1e3 for m in ms]}), flush=True)
    L.traj_debug_fused_waves(0)


if __name__ == "__main__":
    main()
