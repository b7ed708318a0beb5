"""ctypes binding of oracle/build/libtraj_oracle.so (TEST INFRASTRUCTURE ONLY).

The C restatement it binds is documented in oracle/traj_oracle.h; every function
there cites the reference file:line it follows (MPC/mpc_6stati.py, MPC/main.py).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libtraj_oracle.so")

STATUS_NAMES = {
    0: "optimal",
    1: "optimal_inaccurate",
    2: "user_limit",
    3: "infeasible",
    4: "infeasible_inaccurate",
    5: "unbounded",
    6: "solver_error",
}

_D = C.POINTER(C.c_double)
_I = C.POINTER(C.c_int)


class OrcParams(C.Structure):
    _fields_ = [(k, C.c_double) for k in (
        "Cm1", "Cm2", "Cr0", "Cr2", "Br", "Cr", "Dr", "Bf", "Cf", "Df", "m", "Iz", "lf", "lr", "g",
        "maxAlpha", "vx_zero")]


class OrcCfg(C.Structure):
    _fields_ = [
        ("N", C.c_int), ("Ts", C.c_double),
        ("q_c", C.c_double), ("q_phi", C.c_double), ("q_vx", C.c_double),
        ("R", C.c_double * 4), ("Rd", C.c_double * 4),
        ("u_lo", C.c_double * 2), ("u_hi", C.c_double * 2),
        ("du_lo", C.c_double * 2), ("du_hi", C.c_double * 2),
        ("has_x_lo", C.c_int), ("has_x_hi", C.c_int),
        ("x_lo", C.c_double * 6), ("x_hi", C.c_double * 6),
        ("eps_abs", C.c_double), ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double),
        ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double), ("delta", C.c_double),
        ("max_iter", C.c_int), ("check_interval", C.c_int), ("scaling_iters", C.c_int),
        ("polish", C.c_int), ("polish_refine_iter", C.c_int), ("adaptive_rho", C.c_int),
        ("adaptive_rho_tol", C.c_double),
        ("polish_mode", C.c_int), ("polish_max_pass", C.c_int), ("cert_tol", C.c_double),
        ("polish_max_rounds", C.c_int), ("warm_start", C.c_int),
        ("solver", C.c_int), ("ipm_max_iter", C.c_int), ("ipm_tol", C.c_double),
    ]


class OrcInfo(C.Structure):
    _fields_ = [("status", C.c_int), ("iters", C.c_int), ("polished", C.c_int),
                ("prim_res", C.c_double), ("dual_res", C.c_double), ("rho_final", C.c_double),
                ("objective", C.c_double)]


class OrcPath(C.Structure):
    _fields_ = [("kind", C.c_int), ("nk", C.c_int), ("c", C.c_double * 4), ("xk", _D), ("coef", _D)]


_lib = None


def build(force: bool = False) -> str:
    """Compile the oracle with its Makefile (gcc); returns the .so path."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.orc_default_params.argtypes = [C.POINTER(OrcParams)]
        L.orc_default_cfg.argtypes = [C.POINTER(OrcCfg), C.c_int, C.c_double]
        L.orc_tire_forces.argtypes = [C.POINTER(OrcParams), _D, _D, _D]
        L.orc_f_cont.argtypes = [C.POINTER(OrcParams), _D, _D, _D]
        L.orc_numerical_jacobian.argtypes = [C.POINTER(OrcParams), _D, _D, C.c_double, C.c_double, _D, _D, _D]
        L.orc_linearize_discretize.argtypes = [C.POINTER(OrcParams), _D, _D, C.c_double, _D, _D, _D]
        L.orc_lateral_error.argtypes = [C.c_double] * 5
        L.orc_lateral_error.restype = C.c_double
        L.orc_nominal_rollout.argtypes = [C.POINTER(OrcParams), _D, _D, C.c_int, C.c_double, _D]
        L.orc_mpc_step.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), _D, _D, _D, _D, _D, _D, _D,
                                   C.POINTER(OrcInfo)]
        L.orc_mpc_step.restype = C.c_int
        L.orc_mpc_step_batch.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), C.c_int, _D, _D, _D, _D, _D,
                                         _I, _D, _D, _D, _I, _I, C.c_int]
        L.orc_mpc_step_batch_warm.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), C.c_int, _D, _D, _D, _D, _D,
                                              _I, _D, _I, _I, _I, C.c_int]
        L.orc_qp_exact.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), _D, _D, _D, _D, _D, _D]
        L.orc_qp_exact.restype = C.c_int
        L.orc_qp_ipm.argtypes = [C.POINTER(OrcCfg), _D, _D, _D, _D, _D, _D, _D, _D, _D, _D, C.POINTER(OrcInfo)]
        L.orc_qp_ipm.restype = C.c_int
        L.orc_d_steady_state.argtypes = [C.POINTER(OrcParams), C.c_double]
        L.orc_d_steady_state.restype = C.c_double
        L.orc_vref_ramp.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, _D]
        L.orc_path_eval.argtypes = [C.POINTER(OrcPath), C.c_double, _D, _D]
        L.orc_ref_window.argtypes = [C.POINTER(OrcPath), C.c_double, C.c_int, C.c_double, _D, _D]
        L.orc_spline_natural.argtypes = [C.c_int, _D, _D, _D]
        L.orc_closed_loop.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), C.POINTER(OrcPath), _D, _D, _D,
                                      C.c_int, _D, _D, _I, _I]
        L.orc_closed_loop_batch.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcCfg), C.POINTER(OrcPath), C.c_int,
                                            _D, _D, _D, C.c_int, _D, _D, _I, _I, C.c_int]
        L.orc_set_tire_sine.argtypes = [C.c_int]
        L.orc_set_tire_sine.restype = C.c_int
        L.orc_tire_sin.argtypes = [C.c_double]
        L.orc_tire_sin.restype = C.c_double
        _lib = L
    return _lib


def set_tire_sine(mode: int) -> int:
    """0: libm sin in the tire forces (default, pinned by the reference fixtures); 1: the HIP path's bounded-range
    polynomial (physics.h tire_sin_poly, same coefficients and fma order).  Returns the previous mode."""
    return int(lib().orc_set_tire_sine(int(mode)))


def tire_sin(z) -> np.ndarray:
    """The oracle's tire sine in the current mode, elementwise."""
    f = lib().orc_tire_sin
    return np.array([f(float(v)) for v in np.asarray(z, np.float64).reshape(-1)]).reshape(np.shape(z))


class tire_sine:
    """Context manager: `with tire_sine(1): ...` runs the oracle with the HIP path's tire sine, then restores."""

    def __init__(self, mode: int):
        self.mode = mode

    def __enter__(self):
        self.prev = set_tire_sine(self.mode)
        return self

    def __exit__(self, *exc):
        set_tire_sine(self.prev)
        return False


def _dp(a):
    return a.ctypes.data_as(_D) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(_I) if a is not None else None


def _f64(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    if shape is not None:
        a = a.reshape(shape)
    return a


# --------------------------------------------------------------- params/config

def params(overrides: dict | None = None) -> OrcParams:
    p = OrcParams()
    lib().orc_default_params(C.byref(p))
    for k, v in (overrides or {}).items():
        if hasattr(p, k):
            setattr(p, k, float(v))
    return p


def cfg(N=20, Ts=0.02, q_c=6.0, q_phi=0.5, q_vx=0.5, R=None, Rd=None, u_bounds=((-1.0, 1.0), (-0.6, 0.6)),
        du_bounds=((-0.5, 0.5), (-0.3, 0.3)), x_lo=None, x_hi=None, **solver) -> OrcCfg:
    c = OrcCfg()
    lib().orc_default_cfg(C.byref(c), int(N), float(Ts))
    c.q_c, c.q_phi, c.q_vx = float(q_c), float(q_phi), float(q_vx)
    R = np.diag([0.02, 2.0]) if R is None else np.asarray(R, dtype=np.float64).reshape(2, 2)
    Rd = np.diag([0.01, 5.0]) if Rd is None else np.asarray(Rd, dtype=np.float64).reshape(2, 2)
    for i in range(4):
        c.R[i] = R.flat[i]
        c.Rd[i] = Rd.flat[i]
    for ch in range(2):
        c.u_lo[ch], c.u_hi[ch] = map(float, u_bounds[ch])
        c.du_lo[ch], c.du_hi[ch] = map(float, du_bounds[ch])
    if x_lo is not None:
        c.has_x_lo = 1
        for i, v in enumerate(np.asarray(x_lo, dtype=np.float64).reshape(6)):
            c.x_lo[i] = v
    if x_hi is not None:
        c.has_x_hi = 1
        for i, v in enumerate(np.asarray(x_hi, dtype=np.float64).reshape(6)):
            c.x_hi[i] = v
    for k, v in solver.items():
        setattr(c, k, v)
    return c


# --------------------------------------------------------------- physics

def tire_forces(x, u, p=None):
    p = p or params()
    out = np.zeros(3)
    lib().orc_tire_forces(C.byref(p), _dp(_f64(x, 6)), _dp(_f64(u, 2)), _dp(out))
    return out


def f_cont(x, u, p=None):
    p = p or params()
    out = np.zeros(6)
    lib().orc_f_cont(C.byref(p), _dp(_f64(x, 6)), _dp(_f64(u, 2)), _dp(out))
    return out


def numerical_jacobian(x, u, p=None, eps_x=1e-5, eps_u=1e-5):
    p = p or params()
    Jx, Ju, f = np.zeros((6, 6)), np.zeros((6, 2)), np.zeros(6)
    lib().orc_numerical_jacobian(C.byref(p), _dp(_f64(x, 6)), _dp(_f64(u, 2)), eps_x, eps_u, _dp(Jx), _dp(Ju),
                                 _dp(f))
    return Jx, Ju, f


def linearize_discretize(xbar, ubar, Ts, p=None):
    p = p or params()
    A, B, g = np.zeros((6, 6)), np.zeros((6, 2)), np.zeros(6)
    lib().orc_linearize_discretize(C.byref(p), _dp(_f64(xbar, 6)), _dp(_f64(ubar, 2)), float(Ts), _dp(A), _dp(B),
                                   _dp(g))
    return A, B, g


def lateral_error(X, Y, Xr, Yr, phir):
    return lib().orc_lateral_error(float(X), float(Y), float(Xr), float(Yr), float(phir))


def nominal_rollout(x0, u_prev, N, Ts, p=None):
    p = p or params()
    xbar = np.zeros((6, N + 1))
    lib().orc_nominal_rollout(C.byref(p), _dp(_f64(x0, 6)), _dp(_f64(u_prev, 2)), int(N), float(Ts), _dp(xbar))
    return xbar


# --------------------------------------------------------------- MPC step

def mpc_step(x0, u_prev, path_ref, vref, c: OrcCfg, p=None):
    """Returns dict(status, u_cmd, X_opt (6,N+1), U_opt (2,N), objective, iters, polished, prim_res, dual_res)."""
    p = p or params()
    N = c.N
    u_cmd = np.zeros(2)
    X = np.zeros((6, N + 1))
    U = np.zeros((2, N))
    info = OrcInfo()
    lib().orc_mpc_step(C.byref(p), C.byref(c), _dp(_f64(x0, 6)), _dp(_f64(u_prev, 2)),
                       _dp(_f64(path_ref, (N + 1, 3))), _dp(_f64(vref, N + 1)), _dp(u_cmd), _dp(X), _dp(U),
                       C.byref(info))
    return dict(status=info.status, u_cmd=u_cmd, X_opt=X, U_opt=U, objective=info.objective, iters=info.iters,
                polished=info.polished, prim_res=info.prim_res, dual_res=info.dual_res, rho=info.rho_final)


def mpc_step_batch(x0, u_prev, path_ref, vref, c: OrcCfg, p=None, nthreads=0):
    p = p or params()
    N = c.N
    x0 = _f64(x0)
    B = x0.shape[0]
    u_prev = _f64(u_prev, (B, 2))
    path_ref = _f64(path_ref, (B, N + 1, 3))
    vref = _f64(vref, (B, N + 1))
    out = dict(u_cmd=np.zeros((B, 2)), status=np.zeros(B, np.int32), objective=np.zeros(B),
               X_opt=np.zeros((B, 6, N + 1)), U_opt=np.zeros((B, 2, N)), iters=np.zeros(B, np.int32),
               polished=np.zeros(B, np.int32))
    lib().orc_mpc_step_batch(C.byref(p), C.byref(c), B, _dp(x0), _dp(u_prev), _dp(path_ref), _dp(vref),
                             _dp(out["u_cmd"]), _ip(out["status"]), _dp(out["objective"]), _dp(out["X_opt"]),
                             _dp(out["U_opt"]), _ip(out["iters"]), _ip(out["polished"]), int(nthreads))
    return out


def mpc_step_batch_warm(x0, u_prev, path_ref, vref, rho, valid, c: OrcCfg, p=None, nthreads=0):
    """mpc_step_batch with each instance's warm start (traj_oracle.c orc_mpc_step_batch_warm): rho [B] and valid [B]
    are the rho carried from the instance's previous step; returns the outputs with the updated rho / valid."""
    p = p or params()
    N = c.N
    x0 = _f64(x0)
    B = x0.shape[0]
    u_prev = _f64(u_prev, (B, 2))
    path_ref = _f64(path_ref, (B, N + 1, 3))
    vref = _f64(vref, (B, N + 1))
    rho = np.ascontiguousarray(rho, dtype=np.float64).copy()
    valid = np.ascontiguousarray(valid, dtype=np.int32).copy()
    out = dict(u_cmd=np.zeros((B, 2)), status=np.zeros(B, np.int32), iters=np.zeros(B, np.int32),
               polished=np.zeros(B, np.int32))
    lib().orc_mpc_step_batch_warm(C.byref(p), C.byref(c), B, _dp(x0), _dp(u_prev), _dp(path_ref), _dp(vref),
                                  _dp(rho), _ip(valid), _dp(out["u_cmd"]), _ip(out["status"]), _ip(out["iters"]),
                                  _ip(out["polished"]), int(nthreads))
    out["rho"], out["valid"] = rho, valid
    return out


def qp_exact(x0, u_prev, path_ref, vref, c: OrcCfg, p=None):
    """Interior-point solve of the same condensed QP (validation solver). Returns (U_opt (2,N), objective) or None."""
    p = p or params()
    N = c.N
    U = np.zeros((2, N))
    obj = C.c_double(0.0)
    rc = lib().orc_qp_exact(C.byref(p), C.byref(c), _dp(_f64(x0, 6)), _dp(_f64(u_prev, 2)),
                            _dp(_f64(path_ref, (N + 1, 3))), _dp(_f64(vref, N + 1)), _dp(U), C.byref(obj))
    return (U, obj.value) if rc == 0 else None


def qp_ipm(x0, u_prev, path_ref, vref, Ad, Bd, g, c: OrcCfg, xinit=None):
    """The QP half (mpc_6stati.py:180-275) in its sparse form by the structured interior-point method
    (riccati_ipm.c) with the linearization given: Ad [N,6,6], Bd [N,6,2], g [N,6]; xinit [N+1,6] starting
    states (default zeros).  Returns dict(status, U_opt (2,N), X_opt (6,N+1), objective, iters)."""
    N = c.N
    U = np.full((2, N), np.nan)
    X = np.full((6, N + 1), np.nan)
    info = OrcInfo()
    xi = None if xinit is None else _f64(xinit, (N + 1, 6))
    lib().orc_qp_ipm(C.byref(c), _dp(_f64(x0, 6)), _dp(_f64(u_prev, 2)), _dp(_f64(path_ref, (N + 1, 3))),
                     _dp(_f64(vref, N + 1)), _dp(_f64(Ad, (N, 6, 6))), _dp(_f64(Bd, (N, 6, 2))), _dp(_f64(g, (N, 6))),
                     _dp(xi), _dp(U), _dp(X), C.byref(info))
    return dict(status=info.status, U_opt=U, X_opt=X, objective=info.objective, iters=info.iters,
                prim_res=info.prim_res, dual_res=info.dual_res)


# --------------------------------------------------------------- closed loop helpers

def d_steady_state(v, p=None):
    p = p or params()
    return lib().orc_d_steady_state(C.byref(p), float(v))


def vref_ramp(N, Ts, v0=0.8, v_cruise=2.0, tramp=2.0):
    v = np.zeros(N + 1)
    lib().orc_vref_ramp(int(N), float(Ts), float(v0), float(v_cruise), float(tramp), _dp(v))
    return v


class Path:
    """Holds an OrcPath plus the arrays it points to (keeps them alive)."""

    def __init__(self, kind, c=(0.0, 0.0, 0.0, 0.0), xk=None, coef=None):
        self._xk = None if xk is None else _f64(xk)
        self._coef = None if coef is None else _f64(coef)
        self.s = OrcPath()
        self.s.kind = int(kind)
        self.s.nk = 0 if xk is None else len(self._xk)
        for i in range(4):
            self.s.c[i] = float(c[i])
        self.s.xk = _dp(self._xk) if self._xk is not None else None
        self.s.coef = _dp(self._coef) if self._coef is not None else None

    def eval(self, x):
        y, dy = C.c_double(), C.c_double()
        lib().orc_path_eval(C.byref(self.s), float(x), C.byref(y), C.byref(dy))
        return y.value, dy.value


def spline_natural(xk, yk):
    xk, yk = _f64(xk), _f64(yk)
    coef = np.zeros(4 * (len(xk) - 1))
    lib().orc_spline_natural(len(xk), _dp(xk), _dp(yk), _dp(coef))
    return coef


def ref_window(path: Path, x_start, N, Ts, vref):
    out = np.zeros((N + 1, 3))
    lib().orc_ref_window(C.byref(path.s), float(x_start), int(N), float(Ts), _dp(_f64(vref, N + 1)), _dp(out))
    return out


def closed_loop(path: Path, x0, u0, vref, T, c: OrcCfg, p=None):
    p = p or params()
    tx = np.zeros((T + 1, 6))
    tu = np.zeros((T, 2))
    st = np.zeros(T, np.int32)
    it = np.zeros(T, np.int32)
    lib().orc_closed_loop(C.byref(p), C.byref(c), C.byref(path.s), _dp(_f64(x0, 6)), _dp(_f64(u0, 2)),
                          _dp(_f64(vref, c.N + 1)), int(T), _dp(tx), _dp(tu), _ip(st), _ip(it))
    return dict(X=tx, U=tu, status=st, iters=it)


def closed_loop_batch(paths: list, x0, u0, vref, T, c: OrcCfg, p=None, nthreads=0):
    """B closed loops with OpenMP over trajectories; paths is a list of Path."""
    p = p or params()
    B = len(paths)
    arr = (OrcPath * B)(*[pa.s for pa in paths])
    x0 = _f64(x0, (B, 6)); u0 = _f64(u0, (B, 2))
    tx = np.zeros((B, T + 1, 6)); tu = np.zeros((B, T, 2))
    st = np.zeros((B, T), np.int32); it = np.zeros((B, T), np.int32)
    lib().orc_closed_loop_batch(C.byref(p), C.byref(c), arr, B, _dp(x0), _dp(u0), _dp(_f64(vref, c.N + 1)), int(T),
                                _dp(tx), _dp(tu), _ip(st), _ip(it), int(nthreads))
    return dict(X=tx, U=tu, status=st, iters=it)
