"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own code.

Run in the build container only (it reads /root/reference, which does not
exist on the GPU box):  python tests/golden/gen_golden.py

What is taken from the reference (imported read-only from /root/reference/MPC):
  * mpc_6stati.tire_forces / f_cont / numerical_jacobian /
    linearize_discretize / lateral_error  (MPC/mpc_6stati.py:25-117)
  * the nominal rollout loop is the one of mpc_step (mpc_6stati.py:165-172),
    driven with the reference f_cont.
`import cvxpy` (mpc_6stati.py:6) and the default argument `solver=cp.OSQP`
(:141) are evaluated at import; cvxpy is not installed in this image, so a
stub module exposing only `OSQP` is placed in sys.modules.  No cvxpy code path
is executed by anything below.

The QP half of mpc_step (CVXPY + OSQP, :180-262) cannot run here.  Its golden
solutions are produced by an independent solver in this file: the QP is
built in the SPARSE form CVXPY builds (variables X (6,N+1) and U (2,N),
equalities :185-193, inequalities :195-213, objective :217-250) from the
reference's own (Ad, Bd, g), solved by a dense primal-dual interior point
method, then finished by an exact equality-constrained KKT solve on the
identified active set and accepted only if the KKT conditions (stationarity,
feasibility, multiplier signs) hold.  The optimum is unique (R > 0), so any
accurate solver -- OSQP included, when its polish succeeds -- returns it.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

REF_MPC = "/root/reference/MPC"
OUT = os.path.dirname(os.path.abspath(__file__))


def import_reference():
    stub = types.ModuleType("cvxpy")
    stub.OSQP = "OSQP"
    sys.modules.setdefault("cvxpy", stub)
    sys.path.insert(0, REF_MPC)
    import mpc_6stati  # noqa: E402  (reference module)
    return mpc_6stati


# ----------------------------------------------------------------------------- sparse QP

def build_sparse_qp(ref, x0, u_prev, path_ref, vref, N, Ts, params=None, q_c=6.0, q_phi=0.5, q_vx=0.5,
                    R=np.diag([0.02, 2.0]), Rd=np.diag([0.01, 5.0]), u_bounds=((-1.0, 1.0), (-0.6, 0.6)),
                    du_bounds=((-0.5, 0.5), (-0.3, 0.3))):
    """The QP of mpc_6stati.py:180-250 over z = [vec(X) (k-major: X[:,0], X[:,1], ...), vec(U) (k-major)]."""
    p = dict(ref.Params)
    if params:
        p.update(params)
    nx, nu = 6, 2
    NX = nx * (N + 1)
    nz = NX + nu * N
    xi = lambda k, i: nx * k + i          # noqa: E731
    ui = lambda k, j: NX + nu * k + j     # noqa: E731
    # nominal rollout + linearization, exactly as mpc_step (:165-178), with reference functions
    xbar = np.zeros((6, N + 1))
    xbar[:, 0] = x0
    for k in range(N):
        xbar[:, k + 1] = xbar[:, k] + Ts * ref.f_cont(xbar[:, k], u_prev, p)
    lin = [ref.linearize_discretize(xbar[:, k], u_prev, Ts, p) for k in range(N)]
    # equalities E z = e
    E = np.zeros((nx * (N + 1), nz))
    e = np.zeros(nx * (N + 1))
    for i in range(nx):
        E[i, xi(0, i)] = 1.0
        e[i] = x0[i]
    for k in range(N):
        Ad, Bd, g = lin[k]
        for i in range(nx):
            r = nx * (k + 1) + i
            E[r, xi(k + 1, i)] = 1.0
            for jj in range(nx):
                E[r, xi(k, jj)] -= Ad[i, jj]
            for jj in range(nu):
                E[r, ui(k, jj)] -= Bd[i, jj]
            e[r] = g[i]
    # inequalities as two-sided rows l <= A z <= u
    rows, lo, hi = [], [], []
    for k in range(N):
        for j in range(nu):
            a = np.zeros(nz); a[ui(k, j)] = 1.0
            rows.append(a); lo.append(u_bounds[j][0]); hi.append(u_bounds[j][1])
        for j in range(nu):
            a = np.zeros(nz); a[ui(k, j)] = 1.0
            if k == 0:
                rows.append(a); lo.append(du_bounds[j][0] + u_prev[j]); hi.append(du_bounds[j][1] + u_prev[j])
            else:
                a[ui(k - 1, j)] = -1.0
                rows.append(a); lo.append(du_bounds[j][0]); hi.append(du_bounds[j][1])
    A = np.array(rows)
    l, u = np.array(lo), np.array(hi)
    # objective 1/2 z'Qz + c'z + const
    Q = np.zeros((nz, nz))
    c = np.zeros(nz)
    const = 0.0
    Xr, Yr, Pr = path_ref[:, 0], path_ref[:, 1], path_ref[:, 2]
    for k in range(N + 1):
        s, co = np.sin(Pr[k]), np.cos(Pr[k])
        terms = [
            (q_c, {xi(k, 0): s, xi(k, 1): -co}, s * Xr[k] - co * Yr[k]),
            (q_phi, {xi(k, 2): 1.0}, Pr[k]),
            (q_vx, {xi(k, 3): 1.0}, vref[k]),
        ]
        for w, coef, tgt in terms:
            idx = list(coef)
            vals = np.array([coef[i] for i in idx])
            for a_, va in zip(idx, vals):
                c[a_] += -2.0 * w * va * tgt
                for b_, vb in zip(idx, vals):
                    Q[a_, b_] += 2.0 * w * va * vb
            const += w * tgt * tgt
    Rs = 0.5 * (R + R.T)
    Rds = 0.5 * (Rd + Rd.T)
    for k in range(N):
        for a_ in range(nu):
            for b_ in range(nu):
                Q[ui(k, a_), ui(k, b_)] += 2.0 * Rs[a_, b_]
                # dU_k = U_k - U_{k-1} (U_{-1} = u_prev constant)
                Q[ui(k, a_), ui(k, b_)] += 2.0 * Rds[a_, b_]
                if k > 0:
                    Q[ui(k - 1, a_), ui(k - 1, b_)] += 2.0 * Rds[a_, b_]
                    Q[ui(k, a_), ui(k - 1, b_)] -= 2.0 * Rds[a_, b_]
                    Q[ui(k - 1, a_), ui(k, b_)] -= 2.0 * Rds[a_, b_]
    for a_ in range(nu):
        t = Rds[a_] @ u_prev
        c[ui(0, a_)] -= 2.0 * t
        const += u_prev[a_] * t
    return dict(Q=Q, c=c, const=const, E=E, e=e, A=A, l=l, u=u, nz=nz, NX=NX, lin=lin, xbar=xbar)


def solve_ipm(qp, iters=200):
    """Dense Mehrotra predictor-corrector IPM for min 1/2 z'Qz + c'z, Ez = e, Gz <= h."""
    Q, c, E, e = qp["Q"], qp["c"], qp["E"], qp["e"]
    G = np.vstack([qp["A"], -qp["A"]])
    h = np.concatenate([qp["u"], -qp["l"]])
    nz, me, mg = Q.shape[0], E.shape[0], G.shape[0]
    z = np.zeros(nz)
    nu_ = np.zeros(me)
    s = np.maximum(h - G @ z, 1.0)
    lam = np.ones(mg)
    for _ in range(iters):
        rd = Q @ z + c + E.T @ nu_ + G.T @ lam
        re = E @ z - e
        rp = G @ z + s - h
        mu = s @ lam / mg
        if (np.abs(rd).max() < 1e-11 * (1 + np.abs(c).max()) and np.abs(re).max() < 1e-12
                and np.abs(rp).max() < 1e-12 and mu < 1e-13):
            break
        W = lam / s
        K = np.block([[Q + G.T @ (W[:, None] * G), E.T], [E, np.zeros((me, me))]])
        ds_aff = dl_aff = None
        sigma = 0.0
        for pas in range(2):
            rc = -s * lam if pas == 0 else -s * lam + sigma * mu - ds_aff * dl_aff
            rhs1 = -rd - G.T @ ((rc + lam * rp) / s)
            sol = np.linalg.solve(K, np.concatenate([rhs1, -re]))
            dz, dn = sol[:nz], sol[nz:]
            ds = -rp - G @ dz
            dl = (rc - lam * ds) / s
            a = 1.0
            neg = ds < 0
            if neg.any():
                a = min(a, np.min(-s[neg] / ds[neg]))
            neg = dl < 0
            if neg.any():
                a = min(a, np.min(-lam[neg] / dl[neg]))
            if pas == 0:
                mu_aff = (s + a * ds) @ (lam + a * dl) / mg
                sigma = (mu_aff / mu) ** 3
                ds_aff, dl_aff = ds, dl
            else:
                a = min(1.0, 0.99 * a)
                z += a * dz
                nu_ += a * dn
                s += a * ds
                lam += a * dl
    m = qp["A"].shape[0]
    y = lam[:m] - lam[m:]          # y > 0 upper active, y < 0 lower active (OSQP sign convention)
    return z, nu_, y


def exact_kkt(qp, z, y, tol=1e-9):
    """Identify the active set from the IPM point, solve the equality-constrained KKT system exactly
    (dense LU on the sparse-form KKT matrix), and certify.  Returns (z, y, kkt_residuals) or raises."""
    Q, c, E, e, A, l, u = qp["Q"], qp["c"], qp["E"], qp["e"], qp["A"], qp["l"], qp["u"]
    nz, me, m = Q.shape[0], E.shape[0], A.shape[0]
    Az = A @ z
    scale_y = max(1.0, np.abs(y).max())
    act = np.zeros(m, int)
    act[(Az - l < 1e-7) & (y < -1e-9 * scale_y)] = -1
    act[(u - Az < 1e-7) & (y > 1e-9 * scale_y)] = 1
    for _ in range(20):
        ia = np.nonzero(act)[0]
        Aa = A[ia]
        ba = np.where(act[ia] < 0, l[ia], u[ia])
        na = len(ia)
        K = np.block([[Q, E.T, Aa.T], [E, np.zeros((me, me)), np.zeros((me, na))],
                      [Aa, np.zeros((na, me)), np.zeros((na, na))]])
        rhs = np.concatenate([-c, e, ba])
        sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
        z2, ya = sol[:nz], sol[nz + me:]
        Az2 = A @ z2
        y2 = np.zeros(m)
        y2[ia] = ya
        viol_lo = l - Az2
        viol_hi = Az2 - u
        bad_sign = ((act < 0) & (y2 > 1e-9 * scale_y)) | ((act > 0) & (y2 < -1e-9 * scale_y))
        worst = max(viol_lo.max(), viol_hi.max())
        if worst <= 1e-10 and not bad_sign.any():
            stat = Q @ z2 + c + E.T @ sol[nz:nz + me] + A.T @ y2
            res = dict(stationarity=float(np.abs(stat).max()), primal=float(max(worst, 0.0)),
                       equality=float(np.abs(E @ z2 - e).max()), n_active=int(na))
            return z2, y2, res
        # primal-dual active set update
        act = np.where(bad_sign, 0, act)
        act[(viol_lo > 1e-10)] = -1
        act[(viol_hi > 1e-10)] = 1
    raise RuntimeError("active-set refinement did not certify")


def objective_ref(ref, X, U, x0, u_prev, path_ref, vref, N, q_c=6.0, q_phi=0.5, q_vx=0.5,
                  R=np.diag([0.02, 2.0]), Rd=np.diag([0.01, 5.0])):
    """mpc_6stati.py:217-250 evaluated numerically (prob.value includes the constant k=0 terms)."""
    obj = 0.0
    for k in range(N + 1):
        ec = ref.lateral_error(X[0, k], X[1, k], path_ref[k, 0], path_ref[k, 1], path_ref[k, 2])
        obj += q_c * ec ** 2 + q_phi * (X[2, k] - path_ref[k, 2]) ** 2 + q_vx * (X[3, k] - vref[k]) ** 2
        if k == N:
            break
        du = U[:, k] - (u_prev if k == 0 else U[:, k - 1])
        obj += U[:, k] @ R @ U[:, k] + du @ Rd @ du
    return obj


# ----------------------------------------------------------------------------- fixtures

def sample_points(rng, n):
    x = np.stack([rng.uniform(-3, 3, n), rng.uniform(-3, 3, n), rng.uniform(-np.pi, np.pi, n),
                  rng.uniform(0.05, 2.5, n), rng.uniform(-0.3, 0.3, n), rng.uniform(-3, 3, n)], axis=1)
    u = np.stack([rng.uniform(-1, 1, n), rng.uniform(-0.6, 0.6, n)], axis=1)
    # edge cases: vx == 0 (np.sign(0) = 0 -> vx_eff = 0), vx < 0, |vx| == vx_zero, saturated slip angles
    edge_x = np.array([
        [0, 0.5, 0, 0.0, 0.0, 0.0], [0, 0, 0.3, 0.0, 0.1, 0.5], [1, 2, -1, -0.8, 0.05, -0.4],
        [0, 0, 0, 0.3, 0.0, 0.0], [0, 0, 0, -0.3, 0.02, 0.1], [0, 0, 0, 1.0, 0.9, 5.0],
        [0, 0, 0, 1.0, -0.9, -5.0], [0, 0.5, 0, 1.0, 0, 0], [0, 0, 3.0, 0.1, 0.0, 0.0],
        [5, -5, -3.0, 2.0, 0.3, 6.0],
    ])
    edge_u = np.array([[0.2, 0.05], [0.5, 0.6], [-0.3, -0.2], [0.1, 0.0], [0.0, 0.0], [1.0, 0.6],
                       [-1.0, -0.6], [0.2, 0.05], [0.3, 0.1], [0.7, -0.5]])
    return np.vstack([x, edge_x]), np.vstack([u, edge_u])


def gen_physics(ref, rng):
    X, U = sample_points(rng, 256)
    P = ref.Params
    n = len(X)
    tf = np.array([ref.tire_forces(X[i], U[i], P) for i in range(n)])
    fc = np.array([ref.f_cont(X[i], U[i], P) for i in range(n)])
    Jx, Ju, fv = zip(*[ref.numerical_jacobian(ref.f_cont, X[i], U[i], P) for i in range(n)])
    out = dict(x=X, u=U, tire_forces=tf, f_cont=fc, Jx=np.array(Jx), Ju=np.array(Ju), fval=np.array(fv))
    for Ts, tag in ((0.02, "002"), (0.05, "005")):
        A, B, g = zip(*[ref.linearize_discretize(X[i], U[i], Ts, P) for i in range(n)])
        out[f"Ad_{tag}"], out[f"Bd_{tag}"], out[f"g_{tag}"] = np.array(A), np.array(B), np.array(g)
    le_in = rng.uniform(-3, 3, size=(64, 5))
    out["lateral_error_in"] = le_in
    out["lateral_error"] = np.array([ref.lateral_error(*r) for r in le_in])
    # nominal rollouts (:165-172)
    for N in (20, 40):
        for Ts, tag in ((0.02, "002"), (0.05, "005")):
            xb = np.zeros((16, 6, N + 1))
            for i in range(16):
                xb[i, :, 0] = X[i]
                for k in range(N):
                    xb[i, :, k + 1] = xb[i, :, k] + Ts * ref.f_cont(xb[i, :, k], U[i], P)
            out[f"rollout_N{N}_{tag}"] = xb
    out["rollout_x0"] = X[:16]
    out["rollout_u"] = U[:16]
    return out


def ref_window_parabola(x_start, N, Ts, vref, a=0.1):
    """MPC/main.py:51-68 (parabola y = a x^2; the reference uses a = 0.1)."""
    xs = np.zeros(N + 1)
    xs[0] = x_start
    for k in range(N):
        xs[k + 1] = xs[k] + vref[k] * Ts
    return np.stack([xs, a * xs ** 2, np.arctan(2 * a * xs)], axis=1)


def gen_qp(ref, rng, N, Ts, count):
    recs = {k: [] for k in ("x0", "u_prev", "path_ref", "vref", "U_opt", "X_opt", "objective", "stationarity",
                            "n_active", "Ad", "Bd", "g")}
    t = np.arange(N + 1) * Ts
    vref0 = 0.8 + (2.0 - 0.8) * np.clip(t / 2.0, 0.0, 1.0)   # main.py:28-32
    made = 0
    while made < count:
        x0 = np.array([rng.uniform(-2, 2), rng.uniform(-2, 2), rng.uniform(-0.3, 0.3), rng.uniform(0.4, 1.5),
                       rng.uniform(-0.05, 0.05), rng.uniform(-1, 1)])
        u_prev = np.array([rng.uniform(-0.2, 0.5), rng.uniform(-0.3, 0.3)])
        a = rng.uniform(0.05, 0.15)
        path_ref = ref_window_parabola(x0[0], N, Ts, vref0, a)
        path_ref[:, 1] += rng.uniform(-1, 1)
        if made == 0:   # the main.py initial condition (:20-22, :77)
            x0 = np.array([0.0, 0.5, 0.0, 1.0, 0.0, 0.0])
            d_ss = (ref.Params["Cr0"] + ref.Params["Cr2"] * 1.0) / (ref.Params["Cm1"] - ref.Params["Cm2"] * 1.0)
            u_prev = np.array([d_ss, 0.0])
            path_ref = ref_window_parabola(x0[0], N, Ts, vref0, 0.1)
        qp = build_sparse_qp(ref, x0, u_prev, path_ref, vref0, N, Ts)
        z, nu_, y = solve_ipm(qp)
        try:
            z2, y2, res = exact_kkt(qp, z, y)
        except RuntimeError:
            continue
        NX = qp["NX"]
        X = z2[:NX].reshape(N + 1, 6).T
        U = z2[NX:].reshape(N, 2).T
        recs["x0"].append(x0); recs["u_prev"].append(u_prev); recs["path_ref"].append(path_ref)
        recs["vref"].append(vref0); recs["U_opt"].append(U); recs["X_opt"].append(X)
        recs["objective"].append(objective_ref(ref, X, U, x0, u_prev, path_ref, vref0, N))
        recs["stationarity"].append(res["stationarity"]); recs["n_active"].append(res["n_active"])
        recs["Ad"].append(np.array([L[0] for L in qp["lin"]]))
        recs["Bd"].append(np.array([L[1] for L in qp["lin"]]))
        recs["g"].append(np.array([L[2] for L in qp["lin"]]))
        made += 1
    return {k: np.array(v) for k, v in recs.items()}


def main():
    ref = import_reference()
    rng = np.random.default_rng(20261015)
    phys = gen_physics(ref, rng)
    np.savez_compressed(os.path.join(OUT, "physics.npz"), **phys)
    for N, Ts, cnt in ((20, 0.05, 32), (20, 0.02, 16), (40, 0.05, 8), (40, 0.02, 8)):
        q = gen_qp(ref, rng, N, Ts, cnt)
        tag = f"qp_N{N}_Ts{int(round(Ts * 100)):03d}"
        np.savez_compressed(os.path.join(OUT, tag + ".npz"), N=N, Ts=Ts, **q)
        print(tag, "max stationarity", q["stationarity"].max(), "active", q["n_active"].tolist())
    # known-answer anchors quoted by SURVEY.md 8(c)
    xk, uk = np.array([0, .5, 0, 1, 0, 0.]), np.array([.2, .05])
    A, B, g = ref.linearize_discretize(xk, uk, 0.05, ref.Params)
    np.savez(os.path.join(OUT, "anchors.npz"), x=xk, u=uk, f=ref.f_cont(xk, uk, ref.Params), Ad=A, Bd=B, g=g)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
