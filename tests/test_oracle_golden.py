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


def test_tire_sine_poly_vs_libm_and_fixtures(oracle_lib):
    """The HIP path's Pacejka sine (physics.h tire_sin_poly, restated in the oracle as tire_sine mode 1) against
    libm's sine -- the reference's numpy sin: within 2 ulp over the whole range the tire argument C atan(B alpha) can
    take, libm's own value outside it, and the reference fixtures' tire forces / f to the same 1e-13 / 1e-12 bars as
    the libm oracle.  This bounds the one physics difference between the GPU and the reference's libm sine; the GPU
    parity gates run the oracle with the polynomial (tests/test_gpu_parity.py)."""
    O = oracle_lib
    z = np.concatenate([np.linspace(-np.pi / 2, np.pi / 2, 200001), np.random.default_rng(0).uniform(-1.6, 1.6, 50000),
                        [0.0, -0.0, 1e-300, -1e-300, 1e-8, np.pi / 2, -np.pi / 2]])
    with O.tire_sine(1):
        sp = O.tire_sin(z)
        ph = _load("physics")
        tf = np.array([O.tire_forces(x, u) for x, u in zip(ph["x"], ph["u"])])
        fc = np.array([O.f_cont(x, u) for x, u in zip(ph["x"], ph["u"])])
    sl = np.sin(z)
    ulp = np.spacing(np.abs(sl))
    inside = np.abs(z) <= np.pi / 2
    assert (np.abs(sp - sl)[inside] <= 2 * ulp[inside]).all(), (np.abs(sp - sl) / ulp)[inside].max()
    assert np.array_equal(sp[~inside], sl[~inside])
    # (z = -0: the polynomial's fma returns +0 where libm returns -0 -- the same zero force; the GPU does the same)
    assert (sp[z == 0] == 0.0).all()
    np.testing.assert_allclose(tf, ph["tire_forces"], rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(fc, ph["f_cont"], rtol=1e-12, atol=1e-12)
    assert O.set_tire_sine(0) == 0   # the context manager restored the default (libm)


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


@pytest.mark.parametrize("f", QP_FILES)
def test_sparse_structured_ipm_vs_golden(oracle_lib, f):
    """Sparse-form QP (X and U as variables, dynamics as equalities -- the form the reference hands to
    CVXPY, mpc_6stati.py:180-250) solved by the oracle's Riccati-factorized interior point method
    (oracle/riccati_ipm.c) from the reference's own A, B, g: the same unique optimum as the golden."""
    O = oracle_lib
    g = _load(f)
    N, Ts = int(g["N"]), float(g["Ts"])
    c = O.cfg(N=N, Ts=Ts, ipm_tol=1e-12, ipm_max_iter=100)
    for i in range(len(g["x0"])):
        r = O.qp_ipm(g["x0"][i], g["u_prev"][i], g["path_ref"][i], g["vref"][i], g["Ad"][i], g["Bd"][i],
                     g["g"][i], c)
        assert r["status"] == 0 and r["iters"] <= 20
        # interior point: U converges like sqrt(mu) on degenerate active sets -> 1e-4 abs
        assert np.abs(r["U_opt"] - g["U_opt"][i]).max() <= 1e-4
        assert abs(r["objective"] - g["objective"][i]) <= 1e-7 * abs(g["objective"][i])


def test_config3_failures_are_reference_rollout_blowups(oracle_lib):
    """Config 3 (N=40, dt=0.05): every closed-loop step the condensed solver fails on has a REFERENCE
    nominal rollout (mpc_6stati.py:165-172, recorded from the reference's own f_cont by
    tests/golden/gen_hard_qp.py) that reaches |x_bar| >= 1e17 or overflows, so the reference's own QP
    data are non-finite or astronomically scaled there; the oracle's rollout agrees on that, and the
    oracle's condensed solver reproduces the recorded statuses at those states."""
    O = oracle_lib
    g = _load("qp_N40_Ts005_hard")
    N, Ts = int(g["N"]), float(g["Ts"])
    fail = g["failing"] == 1
    assert fail.sum() >= 30 and (~fail).sum() >= 32
    assert float(g["run_fail_min_xbar"]) >= 1e15                  # whole run, not only the kept rows
    assert np.all(g["ref_xbar_max"][fail] >= 1e15)
    assert np.all(g["condensed_status"][fail] >= 2) and np.all(g["condensed_status"][~fail] <= 1)
    c = O.cfg(N=N, Ts=Ts)
    for i in range(len(g["x0"])):
        if not np.isfinite(g["x0"][i]).all():
            continue
        xb = O.nominal_rollout(g["x0"][i], g["u_prev"][i], N, Ts)
        m = np.abs(xb).max() if np.isfinite(xb).all() else np.inf
        # both rollouts are the same float64 recurrence: finite together, and the same order of magnitude
        assert np.isfinite(m) == np.isfinite(g["ref_xbar_max"][i])
        if np.isfinite(m):
            assert abs(np.log10(m) - np.log10(g["ref_xbar_max"][i])) < 1.0
        r = O.mpc_step(g["x0"][i], g["u_prev"][i], g["path_ref"][i], g["vref"][i], c)
        assert r["status"] == g["condensed_status"][i]
        if fail[i]:
            assert np.array_equal(r["u_cmd"], g["u_prev"][i])     # mpc_6stati.py:257-262 fallback
    # controls: where the condensed solver's exact mode CERTIFIES its point (KKT at 1e-9), it and the
    # sparse form (IPM) reach the same optimum.  Uncertified ADMM points (OSQP's polish accepts by a
    # residual comparison) can be far from it at this conditioning: DESIGN.md "Config 3".
    ok = (~fail) & (g["ipm_status"] == 0) & (g["ref_xbar_max"] < 1e3)
    assert ok.sum() >= 32
    cx = O.cfg(N=N, Ts=Ts, polish_mode=1)
    ncert = 0
    for i in np.where(ok)[0]:
        r = O.mpc_step(g["x0"][i], g["u_prev"][i], g["path_ref"][i], g["vref"][i], cx)
        if r["polished"] > 0:
            ncert += 1
            assert np.abs(r["u_cmd"] - g["U_opt"][i][:, 0]).max() <= 1e-4
    assert ncert >= 16
