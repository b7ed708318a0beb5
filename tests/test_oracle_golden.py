"""The CPU oracle (oracle/) against the fixtures generated from the REFERENCE's own code
(tests/golden/gen_golden.py): physics/linearization pinned to MPC/mpc_6stati.py outputs, QP
solutions pinned to an independent sparse-form (CVXPY-shaped) KKT-certified solve."""
import numpy as np
import pytest

GOLD = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden")


def _load(name):
    return np.load(f"{GOLD}/{name}.npz")


def test_known_answer_anchors(oracle_lib):
    """SURVEY.md 8(c) anchors measured from the reference."""
    O = oracle_lib
    a = _load("anchors")
    np.testing.assert_allclose(O.f_cont(a["x"], a["u"]), a["f"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(O.f_cont([0, .5, 0, 1, 0, 0], [.2, .05]),
                               [1, 0, 0, -0.17368083, 0.71692105, 30.66255866], rtol=0, atol=5e-8)
    A, B, g = O.linearize_discretize(a["x"], a["u"], 0.05)
    assert abs(A[5, 4] - 14.203684) < 1e-6 and abs(A[5, 5] + 1.334158) < 1e-6
    assert abs(B[5, 1] - 30.010969) < 1e-6 and abs(g[3] + 0.047693) < 1e-6


def test_physics_vs_reference(oracle_lib):
    O = oracle_lib
    ph = _load("physics")
    X, U = ph["x"], ph["u"]
    tf = np.array([O.tire_forces(x, u) for x, u in zip(X, U)])
    fc = np.array([O.f_cont(x, u) for x, u in zip(X, U)])
    np.testing.assert_allclose(tf, ph["tire_forces"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(fc, ph["f_cont"], rtol=1e-12, atol=1e-12)
    J = [O.numerical_jacobian(x, u) for x, u in zip(X, U)]
    Jx = np.array([j[0] for j in J]); Ju = np.array([j[1] for j in J])
    # central differences amplify last-ulp libm differences by 1/(2 eps) = 5e4
    assert (np.abs(Jx - ph["Jx"]) / (1 + np.abs(ph["Jx"]))).max() < 1e-8
    assert (np.abs(Ju - ph["Ju"]) / (1 + np.abs(ph["Ju"]))).max() < 1e-8
    for Ts, tag in ((0.02, "002"), (0.05, "005")):
        L = [O.linearize_discretize(x, u, Ts) for x, u in zip(X, U)]
        for j, nm in enumerate(("Ad", "Bd", "g")):
            a = np.array([l[j] for l in L]); b = ph[f"{nm}_{tag}"]
            assert (np.abs(a - b) / (1 + np.abs(b))).max() < 1e-9, (nm, tag)
    le = np.array([O.lateral_error(*r) for r in ph["lateral_error_in"]])
    np.testing.assert_allclose(le, ph["lateral_error"], rtol=1e-14, atol=1e-15)


@pytest.mark.parametrize("N", [20, 40])
@pytest.mark.parametrize("tag", ["002", "005"])
def test_nominal_rollout_vs_reference(oracle_lib, N, tag):
    O = oracle_lib
    ph = _load("physics")
    Ts = 0.02 if tag == "002" else 0.05
    for i in range(16):
        xb = O.nominal_rollout(ph["rollout_x0"][i], ph["rollout_u"][i], N, Ts)
        ref = ph[f"rollout_N{N}_{tag}"][i]
        assert (np.abs(xb - ref) / (1 + np.abs(ref))).max() < 1e-9


QP_FILES = ["qp_N20_Ts005", "qp_N20_Ts002", "qp_N40_Ts005", "qp_N40_Ts002"]


@pytest.mark.parametrize("f", QP_FILES)
def test_ipm_validation_solver_vs_golden(oracle_lib, f):
    """Condensed-form interior point (oracle) vs the sparse-form golden optimum: same unique QP."""
    O = oracle_lib
    g = _load(f)
    N, Ts = int(g["N"]), float(g["Ts"])
    c = O.cfg(N=N, Ts=Ts)
    for i in range(len(g["x0"])):
        r = O.qp_exact(g["x0"][i], g["u_prev"][i], g["path_ref"][i], g["vref"][i], c)
        assert r is not None
        # objective is well conditioned; U is not (cond(H) up to ~1e9 at N=40, dt=0.05)
        assert abs(r[1] - g["objective"][i]) <= 1e-7 * abs(g["objective"][i])


@pytest.mark.parametrize("f", QP_FILES)
def test_oracle_mpc_step_vs_golden(oracle_lib, f):
    """Oracle mpc_step (exact polish) vs golden: objective always; U where the KKT certificate holds."""
    O = oracle_lib
    g = _load(f)
    N, Ts = int(g["N"]), float(g["Ts"])
    r = O.mpc_step_batch(g["x0"], g["u_prev"], g["path_ref"], g["vref"], O.cfg(N=N, Ts=Ts, polish_mode=1))
    assert (r["status"] <= 1).all()
    dobj = np.abs(r["objective"] - g["objective"]) / np.abs(g["objective"])
    assert dobj.max() < (1e-5 if N == 40 and Ts == 0.05 else 1e-7)
    cert = r["polished"] > 0
    assert cert.mean() >= (0.5 if N == 40 else 0.9)
    dU = np.abs(r["U_opt"] - g["U_opt"]).max(axis=(1, 2))
    tol = 1e-4 if Ts == 0.05 else 1e-6
    assert dU[cert].max() < tol
    dX = np.abs(r["X_opt"] - g["X_opt"]).max(axis=(1, 2))
    assert dX[cert].max() < 10 * tol


def test_oracle_osqp_polish_mode(oracle_lib):
    """OSQP-faithful mode (single polish): exact optimum when the polish is accepted."""
    O = oracle_lib
    g = _load("qp_N20_Ts002")
    r = O.mpc_step_batch(g["x0"], g["u_prev"], g["path_ref"], g["vref"], O.cfg(N=20, Ts=0.02))
    pol = r["polished"] > 0
    assert pol.mean() > 0.9
    assert np.abs(r["U_opt"] - g["U_opt"]).max(axis=(1, 2))[pol].max() < 1e-8


def test_infeasible_and_nonfinite(oracle_lib):
    O = oracle_lib
    N, Ts = 20, 0.05
    c = O.cfg(N=N, Ts=Ts)
    x0 = np.array([0, 0.5, 0, 1.0, 0, 0])
    v = O.vref_ramp(N, Ts)
    pr = O.ref_window(O.Path(0, (0, 0, 0.1, 0)), 0.0, N, Ts, v)
    # u_prev outside the box by more than one rate step -> U_0 infeasible (mpc_6stati.py:195-206)
    r = O.mpc_step(x0, [2.0, 0.0], pr, v, c)
    assert r["status"] == 3 and np.allclose(r["u_cmd"], [2.0, 0.0])
    pr2 = pr.copy(); pr2[3, 1] = np.nan
    r = O.mpc_step(x0, [0.1, 0.0], pr2, v, c)
    assert r["status"] == 6 and np.allclose(r["u_cmd"], [0.1, 0.0])
