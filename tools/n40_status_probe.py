"""Closed loop at N=40 on mixed references (BASELINE.json configs[2], dt = 0.05): where the GPU
reports non-optimal statuses, re-solve those steps with the oracle from the GPU's own states and
compare (SURVEY.md 8(d) gate (1)).  python tools/n40_status_probe.py [B] [T]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle as O  # noqa: E402  (checker)
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T = int(sys.argv[2]) if len(sys.argv) > 2 else 60
N, Ts = 40, 0.05
O.build()
w = make_workload(B, N, Ts, kind="mixed", seed=0)
paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
cfg = TB.config_struct(N=N, Ts=Ts, warm_start=0)
res = {k: v.cpu().numpy() for k, v in TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, cfg).items()}
st = res["status"]                                       # [T, B]
print("status histogram over the run:", np.bincount(st.reshape(-1), minlength=7).tolist())
vr = np.tile(w["vref"], (B, 1))
agree = tot = 0
first = None
for t in range(T):
    if (st[t] <= 1).all():
        continue
    xt = res["X"][:, t]
    ut = res["U"][:, t - 1] if t > 0 else w["u0"]
    prt = TB.ref_window_batch(paths, xt[:, 0], vr, N, Ts).cpu().numpy()
    ro = O.mpc_step_batch(xt, ut, prt, vr, O.cfg(N=N, Ts=Ts))
    bad = st[t] > 1
    agree += int((ro["status"][bad] == st[t][bad]).sum())
    tot += int(bad.sum())
    if first is None:
        first = t
        i = int(np.flatnonzero(bad)[0])
        print(f"t={t} instance {i}: gpu status {st[t][i]}, oracle {ro['status'][i]}, state {xt[i]}")
print(f"non-optimal GPU statuses re-solved by the oracle: {agree}/{tot} identical")
