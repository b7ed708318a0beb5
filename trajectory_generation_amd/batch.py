"""Batched, device-resident API over libtrajmpc.so (torch.cuda tensors in, torch.cuda tensors out).

Every function here launches HIP kernels through the C ABI (include/trajmpc.h); PyTorch only
provides device memory and the current stream.  There is no CPU fallback.

Reference correspondence (DorianaG01/trajectory_generation):
  f_cont_batch / tire_forces_batch / numerical_jacobian_batch /
  linearize_discretize_batch / lateral_error_batch   MPC/mpc_6stati.py:25-117
  mpc_step_batch                                     MPC/mpc_6stati.py:120-275, B instances at once
  mpc_qp_batch                                       the QP half :180-275 with caller (A, B, g)
  ref_window_batch / PathSet                         MPC/main.py:51-68 (geometry: DESIGN.md)
  closed_loop_step / run_closed_loop                 MPC/main.py:85-101, B trajectories at once
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import MpcConfig, Paths, VehicleParams

REFERENCE_PARAMS = {
    "Cm1": 0.287, "Cm2": 0.0545, "Cr0": 0.0518, "Cr2": 0.00035,
    "Br": 3.3852, "Cr": 1.2691, "Dr": 0.1737, "Bf": 2.579, "Cf": 1.2, "Df": 0.192,
    "m": 0.041, "Iz": 27.8e-6, "lf": 0.029, "lr": 0.033, "g": 9.81, "maxAlpha": 0.6, "vx_zero": 0.3,
}


def require_gpu(device=None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("trajectory_generation_amd needs a ROCm GPU (MI355X); there is no CPU fallback")
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def params_struct(params: dict | VehicleParams | None = None) -> VehicleParams:
    if isinstance(params, VehicleParams):
        return params
    p = _lib.default_params()
    for k, v in (params or {}).items():
        if k in REFERENCE_PARAMS:
            setattr(p, k, float(v))
    return p


def config_struct(N=20, Ts=0.02, q_c=6.0, q_phi=0.5, q_vx=0.5, R=None, Rd=None,
                  u_bounds=((-1.0, 1.0), (-0.6, 0.6)), du_bounds=((-0.5, 0.5), (-0.3, 0.3)),
                  x_lo=None, x_hi=None, **solver) -> MpcConfig:
    """mpc_step keyword arguments (mpc_6stati.py:120-143) -> traj_mpc_config."""
    c = _lib.default_config(int(N), float(Ts))
    c.q_c, c.q_phi, c.q_vx = float(q_c), float(q_phi), float(q_vx)
    R = np.diag([0.02, 2.0]) if R is None else np.asarray(R, dtype=np.float64).reshape(2, 2)
    Rd = np.diag([0.01, 5.0]) if Rd is None else np.asarray(Rd, dtype=np.float64).reshape(2, 2)
    for i in range(4):
        c.R[i] = float(R.flat[i])
        c.Rd[i] = float(Rd.flat[i])
    for ch in range(2):
        c.u_lo[ch], c.u_hi[ch] = (float(v) for v in u_bounds[ch])
        c.du_lo[ch], c.du_hi[ch] = (float(v) for v in du_bounds[ch])
    if x_lo is not None:
        c.has_x_lo = 1
        for i, v in enumerate(np.asarray(x_lo, dtype=np.float64).reshape(6)):
            c.x_lo[i] = float(v)
    if x_hi is not None:
        c.has_x_hi = 1
        for i, v in enumerate(np.asarray(x_hi, dtype=np.float64).reshape(6)):
            c.x_hi[i] = float(v)
    for k, v in solver.items():
        if not hasattr(c, k):
            raise TypeError(f"unknown solver setting {k!r}")
        setattr(c, k, v)
    return c


def _dev(x, shape=None, device=None) -> torch.Tensor:
    dev = require_gpu(device)
    t = torch.as_tensor(x, dtype=torch.float64, device=dev)
    if shape is not None:
        t = t.reshape(shape)
    return t.contiguous()


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


# ---------------------------------------------------------------- physics

def tire_forces_batch(x, u, params=None) -> torch.Tensor:
    x = _dev(x, (-1, 6)); u = _dev(u, (-1, 2))
    out = torch.empty((x.shape[0], 3), dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().traj_tire_forces_batch(C.byref(params_struct(params)), x.shape[0], _p(x), _p(u), _p(out),
                                                 _stream()), "traj_tire_forces_batch")
    return out


def f_cont_batch(x, u, params=None) -> torch.Tensor:
    x = _dev(x, (-1, 6)); u = _dev(u, (-1, 2))
    out = torch.empty((x.shape[0], 6), dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().traj_f_cont_batch(C.byref(params_struct(params)), x.shape[0], _p(x), _p(u), _p(out),
                                            _stream()), "traj_f_cont_batch")
    return out


def numerical_jacobian_batch(x, u, params=None, eps_x=1e-5, eps_u=1e-5):
    x = _dev(x, (-1, 6)); u = _dev(u, (-1, 2))
    B = x.shape[0]
    Jx = torch.empty((B, 6, 6), dtype=torch.float64, device=x.device)
    Ju = torch.empty((B, 6, 2), dtype=torch.float64, device=x.device)
    f = torch.empty((B, 6), dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().traj_numerical_jacobian_batch(C.byref(params_struct(params)), B, _p(x), _p(u),
                                                        float(eps_x), float(eps_u), _p(Jx), _p(Ju), _p(f),
                                                        _stream()), "traj_numerical_jacobian_batch")
    return Jx, Ju, f


def linearize_discretize_batch(xbar, ubar, Ts, params=None):
    x = _dev(xbar, (-1, 6)); u = _dev(ubar, (-1, 2))
    B = x.shape[0]
    A = torch.empty((B, 6, 6), dtype=torch.float64, device=x.device)
    Bm = torch.empty((B, 6, 2), dtype=torch.float64, device=x.device)
    g = torch.empty((B, 6), dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().traj_linearize_discretize_batch(C.byref(params_struct(params)), B, float(Ts), _p(x),
                                                          _p(u), _p(A), _p(Bm), _p(g), _stream()),
               "traj_linearize_discretize_batch")
    return A, Bm, g


def lateral_error_batch(X, Y, Xref, Yref, phiref) -> torch.Tensor:
    ts = [_dev(v, (-1,)) for v in (X, Y, Xref, Yref, phiref)]
    out = torch.empty_like(ts[0])
    _lib.check(_lib.lib().traj_lateral_error_batch(ts[0].shape[0], *[_p(t) for t in ts], _p(out), _stream()),
               "traj_lateral_error_batch")
    return out


# ---------------------------------------------------------------- MPC step

def _outputs(B, N, device):
    f64 = dict(dtype=torch.float64, device=device)
    return dict(u_cmd=torch.empty((B, 2), **f64), status=torch.empty(B, dtype=torch.int32, device=device),
                objective=torch.empty(B, **f64), X_opt=torch.empty((B, 6, N + 1), **f64),
                U_opt=torch.empty((B, 2, N), **f64), iters=torch.empty(B, dtype=torch.int32, device=device),
                polished=torch.empty(B, dtype=torch.int32, device=device))


_WS = {}


def _state_bounds(cfg: MpcConfig) -> bool:
    """x_lo / x_hi given with a finite side (mpc_6stati.py:208-213): the general solver runs."""
    return any((cfg.has_x_lo and cfg.x_lo[i] > -1e30) or (cfg.has_x_hi and cfg.x_hi[i] < 1e30) for i in range(6))


# horizons from which the row-split kernel runs (traj_debug_split_min_n; the library default TRAJ_SPLIT_MIN_N)
SPLIT_MIN_N = _lib.SPLIT_MIN_N


def set_split_min_n(n_min: int) -> None:
    """Experiments: run the row-split kernel from horizon n_min on (step and closed loop; 21 .. MAX_N + 1, the latter
    sending 20 < N <= MAX_N back to the capacity-80 kernel).  The workspace sizes do not depend on it."""
    global SPLIT_MIN_N
    _lib.check(_lib.lib().traj_debug_split_min_n(int(n_min)), "traj_debug_split_min_n")
    SPLIT_MIN_N = int(n_min)


def _general(cfg: MpcConfig) -> bool:
    """The step needs caller-owned scratch (traj_mpc_sb_workspace_bytes): state bounds, or a horizon past the hot
    kernels' capacity (MAX_N < N <= MAX_N_GENERAL, include/trajmpc.h's tiers) or routed to the row-split kernel."""
    return _state_bounds(cfg) or cfg.N > _lib.MAX_N


def workspace(B: int, N: int, device, extra_bytes: int = 0, role: str = "closed_loop") -> torch.Tensor:
    """Cached device workspace for B instances of horizon N (traj_mpc_workspace_bytes), plus extra_bytes
    (traj_mpc_sb_workspace_bytes: the state-bound solver's scratch, caller-owned like the rest).

    One buffer per (device, stream, role).  The closed loop keeps state in its workspace between calls (the
    warm-start records, the previous launch's order, the step queue), so the one-shot step / QP entry points
    use a buffer of their own ("step"): a state-bound solve between two closed-loop steps on the same stream
    must not overwrite -- or, by growing the cache, replace -- the closed loop's buffer."""
    nbytes = int(_lib.lib().traj_mpc_workspace_bytes(int(B), int(N))) + int(extra_bytes)
    key = (str(device), torch.cuda.current_stream(device).cuda_stream, role)
    ws = _WS.get(key)
    if ws is None or ws.numel() * 8 < nbytes:
        new = torch.empty((nbytes + 7) // 8, dtype=torch.float64, device=device)
        if ws is not None:
            new[:ws.numel()].copy_(ws)   # (stream-ordered) what the smaller buffer held stays in place
        ws = new
        _WS[key] = ws
    return ws


def mpc_step_batch(x0, u_prev, path_ref, vref, cfg: MpcConfig, params=None, out: dict | None = None) -> dict:
    """B independent mpc_step calls (mpc_6stati.py:120-275) in one launch.

    x0 [B,6], u_prev [B,2], path_ref [B,N+1,3], vref [B,N+1] (float64, any device; moved to the GPU).
    Returns torch.cuda tensors: u_cmd [B,2], status [B] (int codes, see _lib.STATUS_STRINGS),
    objective [B], X_opt [B,6,N+1], U_opt [B,2,N], iters [B], polished [B]."""
    N = cfg.N
    x0 = _dev(x0, (-1, 6))
    B = x0.shape[0]
    dev = x0.device
    u_prev = _dev(u_prev, (B, 2), dev)
    path_ref = _dev(path_ref, (B, N + 1, 3), dev)
    vref = _dev(vref, (B, N + 1), dev)
    o = out if out is not None else _outputs(B, N, dev)
    sb = int(_lib.lib().traj_mpc_sb_workspace_bytes(B, N)) if _general(cfg) else 0
    ws = workspace(B, N, dev, sb, role="step")
    _lib.check(_lib.lib().traj_mpc_step_batch(
        C.byref(params_struct(params)), C.byref(cfg), B, _p(x0), _p(u_prev), _p(path_ref), _p(vref),
        _p(o["u_cmd"]), _p(o["status"]), _p(o["objective"]), _p(o["X_opt"]), _p(o["U_opt"]), _p(o["iters"]),
        _p(o["polished"]), _p(ws), ws.numel() * 8, _stream()), "traj_mpc_step_batch")
    return o


def mpc_qp_batch(x0, u_prev, path_ref, vref, Ad, Bd, g, cfg: MpcConfig, params=None) -> dict:
    """The QP half of mpc_step (:180-275) with the linearization given: Ad [B,N,6,6], Bd [B,N,6,2], g [B,N,6]."""
    N = cfg.N
    x0 = _dev(x0, (-1, 6))
    B = x0.shape[0]
    dev = x0.device
    args = [_dev(u_prev, (B, 2), dev), _dev(path_ref, (B, N + 1, 3), dev), _dev(vref, (B, N + 1), dev),
            _dev(Ad, (B, N, 6, 6), dev), _dev(Bd, (B, N, 6, 2), dev), _dev(g, (B, N, 6), dev)]
    o = _outputs(B, N, dev)
    sb = int(_lib.lib().traj_mpc_sb_workspace_bytes(B, N)) if _general(cfg) else 0
    ws = workspace(0, N, dev, sb, role="step") if sb else None
    _lib.check(_lib.lib().traj_mpc_qp_batch(
        C.byref(params_struct(params)), C.byref(cfg), B, _p(x0), *[_p(a) for a in args],
        _p(o["u_cmd"]), _p(o["status"]), _p(o["objective"]), _p(o["X_opt"]), _p(o["U_opt"]), _p(o["iters"]),
        _p(o["polished"]), _p(ws) if ws is not None else None, sb, _stream()), "traj_mpc_qp_batch")
    return o


# ---------------------------------------------------------------- closed loop (MPC/main.py)

def d_steady_state(v, params=None):
    """MPC/main.py:9-18 (host arithmetic on a scalar: initial u_prev of the closed loop)."""
    p = dict(REFERENCE_PARAMS)
    p.update(params or {})
    return (p["Cr0"] + p["Cr2"] * v ** 2) / (p["Cm1"] - p["Cm2"] * v)


def vref_ramp(N, Ts, v0=0.8, v_cruise=2.0, tramp=2.0) -> np.ndarray:
    """MPC/main.py:28-32 vref_profile_ramp_cruise."""
    t = np.arange(N + 1) * Ts
    return v0 + (v_cruise - v0) * np.clip(t / tramp, 0.0, 1.0)


def spline_natural(xk, yk):
    """Natural cubic spline piece coefficients (a, b, c, d) per interval, as in oracle/ and DESIGN.md."""
    xk = np.asarray(xk, dtype=np.float64)
    yk = np.asarray(yk, dtype=np.float64)
    n = len(xk)
    h = np.diff(xk)
    M = np.zeros(n)
    if n > 2:
        A = np.zeros((n - 2, n - 2))
        rhs = np.zeros(n - 2)
        for i in range(1, n - 1):
            if i > 1:
                A[i - 1, i - 2] = h[i - 1]
            A[i - 1, i - 1] = 2.0 * (h[i - 1] + h[i])
            if i < n - 2:
                A[i - 1, i] = h[i]
            rhs[i - 1] = 6.0 * ((yk[i + 1] - yk[i]) / h[i] - (yk[i] - yk[i - 1]) / h[i - 1])
        M[1:-1] = np.linalg.solve(A, rhs)
    coef = np.zeros((n - 1, 4))
    coef[:, 0] = yk[:-1]
    coef[:, 1] = (yk[1:] - yk[:-1]) / h - h * (2.0 * M[:-1] + M[1:]) / 6.0
    coef[:, 2] = M[:-1] / 2.0
    coef[:, 3] = (M[1:] - M[:-1]) / (6.0 * h)
    return coef


@dataclass
class PathSet:
    """Per-trajectory reference geometry on the device (traj_paths).

    kind 0: y = c0 + c1 x + c2 x^2 + c3 x^3 (parabola of MPC/main.py:64-66: c2 = 0.1)
    kind 1: y = c0 sin(c1 x + c2) + c3      (sinusoid of MPC/README.md:73-76: c0 = 0.5, c1 = 0.5)
    kind 2: natural cubic spline through nk knots (linear extrapolation outside)."""
    kind: torch.Tensor
    pc: torch.Tensor
    nk: torch.Tensor
    xk: torch.Tensor
    coef: torch.Tensor

    @property
    def B(self):
        return self.kind.shape[0]

    def struct(self) -> Paths:
        s = Paths()
        s.kmax = int(self.xk.shape[1])
        s.kind, s.pc, s.nk, s.xk, s.coef = (t.data_ptr() for t in (self.kind, self.pc, self.nk, self.xk, self.coef))
        return s

    @staticmethod
    def build(kinds, pcs, knots=None, device=None) -> "PathSet":
        """kinds [B] ints, pcs [B,4], knots: list of (xk, yk) (None for kind 0/1)."""
        dev = require_gpu(device)
        B = len(kinds)
        kmax = max([2] + [len(k[0]) for k in (knots or []) if k is not None])
        xk = np.zeros((B, kmax))
        coef = np.zeros((B, kmax - 1, 4))
        nk = np.zeros(B, np.int32)
        for b in range(B):
            if kinds[b] == 2:
                kx, ky = knots[b]
                nk[b] = len(kx)
                xk[b, :len(kx)] = kx
                coef[b, :len(kx) - 1] = spline_natural(kx, ky)
        return PathSet(kind=torch.as_tensor(np.asarray(kinds, np.int32), device=dev),
                       pc=torch.as_tensor(np.asarray(pcs, np.float64).reshape(B, 4), device=dev),
                       nk=torch.as_tensor(nk, device=dev), xk=torch.as_tensor(xk, device=dev),
                       coef=torch.as_tensor(coef, device=dev))


def ref_window_batch(paths: PathSet, x_start, vref, N, Ts) -> torch.Tensor:
    """MPC/main.py:51-68 for B trajectories -> path_ref [B,N+1,3]."""
    xs = _dev(x_start, (-1,))
    B = xs.shape[0]
    vr = _dev(vref, (B, N + 1), xs.device)
    out = torch.empty((B, N + 1, 3), dtype=torch.float64, device=xs.device)
    ps = paths.struct()
    _lib.check(_lib.lib().traj_ref_window_batch(C.byref(ps), B, int(N), float(Ts), _p(xs), _p(vr), _p(out),
                                                _stream()), "traj_ref_window_batch")
    return out


def _closed_extra(B: int, cfg: MpcConfig) -> int:
    """Bytes the closed loop needs past traj_mpc_workspace_bytes (traj_closed_loop_workspace_bytes): the long-horizon
    kernel's scratch (MAX_N_SPLIT < N <= MAX_N_LONG), or with state bounds the general solver's plus the step's window
    and u_cmd (one step per launch sequence, as the step entry point)."""
    L = _lib.lib()
    need = int(L.traj_closed_loop_workspace_bytes(C.byref(cfg), int(B)))
    return max(0, need - int(L.traj_mpc_workspace_bytes(int(B), int(cfg.N))))


def closed_loop_step(x, u_prev, paths: PathSet, vref, cfg: MpcConfig, params=None, t=0, hist_x=None, hist_u=None,
                     status=None, iters=None):
    """One step of MPC/main.py:85-101 for all B trajectories; x [B,6], u_prev [B,2] updated in place."""
    B = x.shape[0]
    ps = paths.struct()
    T = hist_u.shape[1] if hist_u is not None else 0
    ws = workspace(B, cfg.N, x.device, _closed_extra(B, cfg))
    _lib.check(_lib.lib().traj_closed_loop_step(
        C.byref(params_struct(params)), C.byref(cfg), C.byref(ps), B, _p(x), _p(u_prev), _p(vref), int(t), int(T),
        _p(hist_x), _p(hist_u), _p(status), _p(iters), _p(ws), ws.numel() * 8, _stream()), "traj_closed_loop_step")


def closed_loop_run(x, u_prev, paths: PathSet, vref, cfg: MpcConfig, params=None, t0=0, steps=1, hist_x=None,
                    hist_u=None, status=None, iters=None, check=True):
    """Steps t0 .. t0+steps-1 of MPC/main.py:85-101 in ONE fused launch (traj_closed_loop_run), bit-identical
    to `steps` closed_loop_step calls; x, u_prev updated in place; status / iters [steps, B].
    check: synchronize and raise RuntimeError if the run lost an instance hand-off (traj_closed_loop_check)."""
    B = x.shape[0]
    ps = paths.struct()
    T = hist_u.shape[1] if hist_u is not None else 0
    ws = workspace(B, cfg.N, x.device, _closed_extra(B, cfg))
    _lib.check(_lib.lib().traj_closed_loop_run(
        C.byref(params_struct(params)), C.byref(cfg), C.byref(ps), B, _p(x), _p(u_prev), _p(vref), int(t0),
        int(steps), int(T), _p(hist_x), _p(hist_u), _p(status), _p(iters), _p(ws), ws.numel() * 8, _stream()),
        "traj_closed_loop_run")
    if check:   # synchronizes: a lost instance hand-off raises instead of returning stale trajectories
        _lib.check(_lib.lib().traj_closed_loop_check(_p(ws), ws.numel() * 8, B, cfg.N, _stream()),
                   "traj_closed_loop_run")


def run_closed_loop(x0, u0, paths: PathSet, vref, T, cfg: MpcConfig, params=None, record=True, fused=True) -> dict:
    """T closed-loop steps (MPC/main.py:85-101) for B trajectories, all on the device: one fused launch
    (closed_loop_run), or one launch sequence per step (fused=False; identical results).

    Returns X [B,T+1,6] (X[:,0] = x0), U [B,T,2], status [T,B], iters [T,B] (torch.cuda)."""
    x = _dev(x0, (-1, 6)).clone()
    B = x.shape[0]
    dev = x.device
    u = _dev(u0, (B, 2), dev).clone()
    vr = _dev(vref, (-1, cfg.N + 1), dev)
    if vr.shape[0] == 1 and B > 1:
        vr = vr.expand(B, cfg.N + 1).contiguous()
    hx = torch.empty((B, T + 1, 6), dtype=torch.float64, device=dev) if record else None
    hu = torch.empty((B, T, 2), dtype=torch.float64, device=dev) if record else None
    if record:
        hx[:, 0] = x
    st = torch.empty((T, B), dtype=torch.int32, device=dev)
    it = torch.empty((T, B), dtype=torch.int32, device=dev)
    if fused:
        closed_loop_run(x, u, paths, vr, cfg, params, 0, T, hx, hu, st, it)
    else:
        for t in range(T):
            closed_loop_step(x, u, paths, vr, cfg, params, t, hx, hu, st[t], it[t])
    return dict(X=hx, U=hu, status=st, iters=it, x=x, u=u)
