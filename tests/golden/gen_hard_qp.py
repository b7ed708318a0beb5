"""Golden fixture for the config-3 steps that end in "Solver Error" / max-iter (tests/golden/qp_N40_Ts005_hard.npz).

Run in the build container only (it reads /root/reference):  python tests/golden/gen_hard_qp.py

BASELINE.json configs[2] (4096 mixed sinusoid/parabola references, N = 40, dt = 0.05) ends 6.3 % of the
round-1 closed-loop steps in "Solver Error".  The question this fixture answers: is that the build's
condensed formulation, or does the REFERENCE's own QP (the sparse form of MPC/mpc_6stati.py:180-250)
already break down at those states?

  1. The C oracle runs the config-3 closed loop (256 mixed trajectories x 60 steps, same workload
     generator as the bench) and records every step's status.
  2. At every step of that run the REFERENCE's own nominal rollout (mpc_6stati.py:165-172, the
     reference f_cont imported from /root/reference) and its linearize_discretize (:175-178) are
     evaluated at the step's (x0, u_prev); max |x_bar|, max |A_k|, max |g_k| and their finiteness are
     recorded for every step.
  3. Rows kept: the FIRST failing step of every trajectory that fails (the state reached along a path on
     which every earlier step was solved to optimality), 32 further failing steps, and 64 optimal steps
     as a control group (16 of them the optimal steps with the largest rollouts).
  4. For failing rows with finite reference data, gen_golden.build_sparse_qp builds the reference's
     sparse QP from the reference's own (A_k, B_k, g_k) and the oracle's structured IPM
     (oracle/riccati_ipm.c, sparse form, Riccati-factorized) tries to solve it; its status is recorded.
     For control rows the same IPM's U_opt is recorded (it equals the condensed optimum).

What it showed (printed at the end; DESIGN.md "Config 3"): every failing step has a reference nominal
rollout that reaches |x_bar| >= 1e17 or overflows to inf/nan -- 40 Euler steps at constant u_prev of the
open-loop-unstable, stiff plant at Ts = 0.05 -- so the reference's QP data (A_k, g_k) are non-finite or
astronomically scaled there; no failing step has a rollout below 1e15, and the controls stay O(1..1e2)
except a handful that the condensed solver still solves.  These are properties of the reference's own
algorithm, shared by both formulations; on non-finite data the reference's CVXPY/OSQP path raises (or
returns solver_error) and `mpc_step` falls back to u_prev, which is what the build returns.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import gen_golden as G  # noqa: E402
import oracle as O  # noqa: E402  (checker)
from trajectory_generation_amd.workload import make_workload  # noqa: E402

N, TS, B, T = 40, 0.05, 256, 60
N_MORE_FAIL, N_CTRL, N_CTRL_BIG = 32, 64, 16


def ref_rollout_lin(ref, x0, up):
    """mpc_6stati.py:165-178 with the reference's own functions; magnitudes, no QP."""
    p = dict(ref.Params)
    xbar = np.zeros((6, N + 1))
    xbar[:, 0] = x0
    with np.errstate(all="ignore"):
        for k in range(N):
            xbar[:, k + 1] = xbar[:, k] + TS * ref.f_cont(xbar[:, k], up, p)
        A, Bm, g = [], [], []
        for k in range(N):
            a, b, c = ref.linearize_discretize(xbar[:, k], up, TS, p)
            A.append(a), Bm.append(b), g.append(c)
    A, Bm, g = np.array(A), np.array(Bm), np.array(g)

    def mag(a):
        return float(np.abs(a).max()) if np.isfinite(a).all() else np.inf
    return xbar, A, Bm, g, mag(xbar), mag(A), mag(g)


def main():
    ref = G.import_reference()
    O.build()
    w = make_workload(B, N, TS, kind="mixed", seed=0)
    paths = [O.Path(int(k), c) for k, c in zip(w["kinds"], w["pcs"])]
    vref = w["vref"]
    res = O.closed_loop_batch(paths, w["x0"], w["u0"], vref, T, O.cfg(N=N, Ts=TS))
    st = res["status"]                                            # [B, T]
    hist = np.bincount(st.reshape(-1), minlength=7)
    print(f"condensed closed loop (oracle): statuses {hist.tolist()} over {B * T} steps")

    def state(b, t):
        return res["X"][b, t], (res["U"][b, t - 1] if t > 0 else w["u0"][b])

    # reference rollout magnitude of every step of the run
    mx = np.zeros((B, T))
    for b in range(B):
        for t in range(T):
            x0, up = state(b, t)
            mx[b, t] = ref_rollout_lin(ref, x0, up)[4] if np.isfinite(x0).all() else np.inf
    fail = st >= 2
    q = lambda a: np.round(np.log10(np.quantile(a, [0, .5, .9, 1])), 1).tolist()  # noqa: E731
    print(f"log10 max|x_bar| (reference rollout): failing steps min/median/p90/max {q(mx[fail])}; "
          f"optimal steps {q(mx[~fail])}")
    print(f"failing steps with a reference rollout below 1e15: {int((mx[fail] < 1e15).sum())} of {int(fail.sum())}; "
          f"optimal steps above 1e6: {int((mx[~fail] > 1e6).sum())}")

    rng = np.random.default_rng(20261016)
    firsts = [(b, int(np.argmax(fail[b]))) for b in np.where(fail.any(1))[0]]
    others = [tuple(i) for i in np.argwhere(fail) if (i[0], i[1]) not in set(firsts)]
    more = [others[i] for i in np.sort(rng.choice(len(others), size=min(N_MORE_FAIL, len(others)), replace=False))]
    okidx = np.argwhere(~fail)
    big = okidx[np.argsort(-mx[~fail])[:N_CTRL_BIG]]
    rest = okidx[rng.choice(len(okidx), size=N_CTRL - N_CTRL_BIG, replace=False)]
    rows = [(b, t, 1) for b, t in firsts] + [(b, t, 0) for b, t in more] + \
           [(int(b), int(t), -1) for b, t in np.concatenate([big, rest])]

    recs = {k: [] for k in ("x0", "u_prev", "path_ref", "vref", "condensed_status", "first_failure", "failing",
                            "ref_xbar_max", "ref_A_max", "ref_g_max", "ref_finite", "ipm_status", "U_opt",
                            "traj", "step")}
    for b, t, kind in rows:
        x0, up = state(b, t)
        pref = O.ref_window(paths[b], x0[0], N, TS, vref)
        xbar, A, Bm, g, mxb, mA, mg = ref_rollout_lin(ref, x0, up)
        finite = bool(np.isfinite(x0).all() and np.isfinite(A).all() and np.isfinite(Bm).all() and np.isfinite(g).all())
        U = np.full((2, N), np.nan)
        ipm = -1
        if finite:
            r = O.qp_ipm(x0, up, pref, vref, A, Bm, g, O.cfg(N=N, Ts=TS, ipm_tol=1e-12, ipm_max_iter=100),
                         xinit=xbar.T)
            ipm = int(r["status"])
            if kind < 0:
                U = r["U_opt"]
        recs["x0"].append(x0); recs["u_prev"].append(up); recs["path_ref"].append(pref); recs["vref"].append(vref)
        recs["condensed_status"].append(int(st[b, t])); recs["first_failure"].append(int(kind == 1))
        recs["failing"].append(int(kind >= 0))
        recs["ref_xbar_max"].append(mxb); recs["ref_A_max"].append(mA); recs["ref_g_max"].append(mg)
        recs["ref_finite"].append(int(finite)); recs["ipm_status"].append(ipm); recs["U_opt"].append(U)
        recs["traj"].append(int(b)); recs["step"].append(int(t))
    out = {k: np.array(v) for k, v in recs.items()}
    np.savez_compressed(os.path.join(HERE, "qp_N40_Ts005_hard.npz"), N=N, Ts=TS, run_status_hist=hist,
                        run_fail_min_xbar=float(mx[fail].min()), **out)
    f = out["failing"] == 1
    print(f"wrote {len(rows)} rows: {int(f.sum())} failing ({int(out['first_failure'].sum())} first failures), "
          f"{int((~f).sum())} optimal controls")
    print(f"failing rows: reference data finite {int(out['ref_finite'][f].sum())}, min max|x_bar| "
          f"{out['ref_xbar_max'][f].min():.3g}, sparse-IPM statuses on finite ones "
          f"{np.bincount(out['ipm_status'][f & (out['ref_finite'] == 1)], minlength=7).tolist()}")
    print(f"control rows: max|x_bar| median {np.median(out['ref_xbar_max'][~f]):.3g}, sparse-IPM statuses "
          f"{np.bincount(out['ipm_status'][~f] + 1, minlength=8).tolist()} (index 0 = not run)")


if __name__ == "__main__":
    main()
