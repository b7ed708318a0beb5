"""Drop-in replacement for the reference module MPC/mpc_6stati.py.

Same public names, signatures, argument meaning, return values and error behaviour as the
reference; every computation runs in the HIP kernels of libtrajmpc.so on the GPU.

  Params                  mpc_6stati.py:9-19
  clamp                   :21-23
  tire_forces             :25-53
  f_cont                  :55-71
  numerical_jacobian      :73-97
  linearize_discretize    :99-109
  lateral_error           :111-117
  mpc_step                :120-275  -> (u_cmd ndarray(2,), status str, info dict)

`mpc_step` keeps the reference's contract:
  * x0 / u_prev reshaped to (6,) / (2,) (numpy errors propagate); path_ref must be (N+1, 3)
    (AssertionError otherwise, :151); vref None -> x0[3], scalar -> filled, else reshaped (N+1,).
  * status in ("optimal", "optimal_inaccurate") -> (U[:,0], status, info) with info keys
    status / objective / X_opt (6,N+1) / U_opt (2,N) / path_ref / vref  (:264-275).
  * any other status -> (u_prev, status, {})  (:261-262); a solver failure ->
    (u_prev, "Solver Error: <Exception>", {})  (:257-259).
  * `solver` is accepted and ignored (the QP is solved by the HIP ADMM); `verbose` is ignored.
  * any horizon up to 256 (the reference takes any N, :125): N <= 40 runs the register-resident hot
    kernels, 40 < N <= 128 the long-horizon kernel, state bounds or N > 128 the general condensed-QP
    solver (same OSQP restatement; see INTEGRATION.md "Horizon tiers").
The QP's optimum is unique (R > 0), so the result is the one OSQP returns when its polish
succeeds; see DESIGN.md "Parity" for the stated tolerances.
"""
from __future__ import annotations

import ctypes as C

import struct

import numpy as np
import torch

from . import batch as _b
from ._lib import STATUS_STRINGS

# Vehicle Parameters (mpc_6stati.py:9-19)
Params = dict(_b.REFERENCE_PARAMS)


def clamp(x, lo, hi):
    """Utility to constrain values within a range (mpc_6stati.py:21-23)."""
    return np.minimum(np.maximum(x, lo), hi)


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy()


class _CallIO:
    """Pinned host staging for the one-trajectory calls of this module (the reference's call shape): the inputs
    go to the device in ONE copy, the kernel writes every output into ONE device buffer, and ONE copy back plus
    one stream synchronization ends the call -- instead of a copy per argument and a synchronizing read per
    output.  Per (device, stream, N); reused across calls (each call synchronizes before it returns)."""

    _cache: dict = {}

    def __init__(self, dev, nin: int, nf: int, ni: int):
        self.h_in = torch.empty(nin, dtype=torch.float64, pin_memory=True)
        self.d_in = torch.empty(nin, dtype=torch.float64, device=dev)
        nio = nf + (ni + 1) // 2          # int32 outputs packed after the doubles
        self.nf = nf
        self.d_out = torch.empty(nio, dtype=torch.float64, device=dev)
        self.h_out = torch.empty(nio, dtype=torch.float64, pin_memory=True)
        self.a_in = self.h_in.numpy()
        self.a_out = self.h_out.numpy()

    @classmethod
    def get(cls, key, dev, nin, nf, ni):
        k = (str(dev), torch.cuda.current_stream(dev).cuda_stream) + tuple(key)
        io = cls._cache.get(k)
        if io is None:
            io = cls._cache[k] = cls(dev, nin, nf, ni)
        return io

    def step_ptrs(self, N: int):
        """The step entry point's argument pointers into d_in / d_out (fixed per buffer; built once)."""
        if getattr(self, "_ptrs", None) is None:
            i, o, d = self.d_in.data_ptr(), self.d_out.data_ptr(), 8
            oi = o + d * self.nf
            self._ptrs = tuple(C.c_void_p(v) for v in (
                i, i + d * 6, i + d * 8, i + d * (8 + 3 * (N + 1)),                       # x0, u_prev, path_ref, vref
                o, oi, o + d * 2, o + d * 3, o + d * (3 + 6 * (N + 1)), oi + 4, oi + 8))  # u_cmd, status, obj, X, U, it, pol
        return self._ptrs

    def send(self):
        self.d_in.copy_(self.h_in, non_blocking=True)

    def abort(self):
        """A launch after send() raised: let the pending H2D copy from h_in finish before anyone writes h_in again."""
        torch.cuda.current_stream(self.d_in.device).synchronize()

    def receive(self):
        self.h_out.copy_(self.d_out, non_blocking=True)
        torch.cuda.current_stream(self.d_out.device).synchronize()
        return self.a_out


_PSD_CACHE: dict = {}
_STRUCT_CACHE: dict = {}


def _frozen(v):
    """A hashable, exact key for an mpc_step argument (arrays by shape and bytes), or None when there is none."""
    if v is None or isinstance(v, (bool, int, str)):
        return ("s", type(v).__name__, v)   # (by type: 1, 1.0 and True hash alike but are different arguments)
    if isinstance(v, float):
        return ("f", struct.pack("<d", v))  # by bits: -0.0 and 0.0 (and NaN payloads) are distinct keys
    if isinstance(v, np.ndarray):
        return ("a", v.shape, v.dtype.str, v.tobytes())
    if isinstance(v, (tuple, list)):
        parts = tuple(_frozen(e) for e in v)
        return None if any(e is None for e in parts) else ("t", parts)
    if isinstance(v, np.generic):
        return ("g", v.dtype.str, v.tobytes())
    return None


def _params_key(p: dict):
    """Exact key of a params dict whose values are all Python floats (the reference's Params and its overrides): the
    sorted names and the values' bits in one pack -- _frozen's key without its per-item recursion.  None otherwise."""
    ks = sorted(p)
    vs = [p[k] for k in ks]
    if not all(type(v) is float for v in vs):
        return None
    return ("pf", tuple(ks), struct.pack("<%dd" % len(vs), *vs))


def _cached_struct(kind, build, *key_parts, key=None):
    """config_struct / params_struct for the same arguments as a previous call: the same ctypes struct (the C side
    copies it at each launch and never writes it).  Arguments without an exact key are built afresh.  key: an exact
    key computed by the caller (replaces the key parts)."""
    if key is not None:
        key = (kind, key)
    else:
        parts = tuple(_frozen(k) for k in key_parts)
        if any(k is None for k in parts):
            return build()
        key = (kind,) + parts
    v = _STRUCT_CACHE.get(key)
    if v is None:
        if len(_STRUCT_CACHE) > 256:
            _STRUCT_CACHE.clear()
        v = _STRUCT_CACHE[key] = build()
    return v


def _is_psd_cached(M: np.ndarray) -> bool:
    k = (M.shape, M.tobytes())
    v = _PSD_CACHE.get(k)
    if v is None:
        if len(_PSD_CACHE) > 64:
            _PSD_CACHE.clear()
        v = _PSD_CACHE[k] = _is_psd(M)
    return v


def tire_forces(x, u, p):
    """(Fy_f, Fy_r, Frx) at x (6,), u (2,) -- mpc_6stati.py:25-53 (HIP kernel)."""
    out = _np(_b.tire_forces_batch(np.asarray(x, np.float64).reshape(1, 6), np.asarray(u, np.float64).reshape(1, 2),
                                   p))[0]
    return out[0], out[1], out[2]


def f_cont(x, u, p):
    """Continuous-time dynamics f(x,u) -> ndarray (6,) -- mpc_6stati.py:55-71 (HIP kernel)."""
    x = np.asarray(x, np.float64).reshape(6)
    u = np.asarray(u, np.float64).reshape(2)
    dev = _b.require_gpu()
    io = _CallIO.get(("f_cont",), dev, 8, 6, 0)
    io.a_in[:6] = x
    io.a_in[6:] = u
    io.send()
    try:
        _b._lib.check(_b._lib.lib().traj_f_cont_batch(C.byref(_b.params_struct(p)), 1, _b._p(io.d_in),
                                                      C.c_void_p(io.d_in.data_ptr() + 48), _b._p(io.d_out),
                                                      _b._stream()), "traj_f_cont_batch")
    except BaseException:
        io.abort()
        raise
    return io.receive()[:6].copy()


def numerical_jacobian(f, x, u, p, eps_x=1e-5, eps_u=1e-5):
    """Central-difference Jacobians (Jx, Ju, f(x,u)) -- mpc_6stati.py:73-97.

    For the model's own f_cont the differences run in the HIP kernel; any other callable f is
    differenced exactly as the reference does, calling f."""
    x = np.asarray(x, np.float64)
    u = np.asarray(u, np.float64)
    if f is f_cont and x.size == 6 and u.size == 2:
        Jx, Ju, fv = _b.numerical_jacobian_batch(x.reshape(1, 6), u.reshape(1, 2), p, eps_x, eps_u)
        return _np(Jx)[0], _np(Ju)[0], _np(fv)[0]
    n, m = x.size, u.size
    Jx = np.zeros((n, n))
    Ju = np.zeros((n, m))
    for i in range(n):
        dx = np.zeros(n); dx[i] = eps_x
        Jx[:, i] = (f(x + dx, u, p) - f(x - dx, u, p)) / (2.0 * eps_x)
    for j in range(m):
        du = np.zeros(m); du[j] = eps_u
        Ju[:, j] = (f(x, u + du, p) - f(x, u - du, p)) / (2.0 * eps_u)
    return Jx, Ju, f(x, u, p)


def linearize_discretize(x_bar, u_bar, Ts, p):
    """(Ad, Bd, g) -- mpc_6stati.py:99-109 (HIP kernel)."""
    A, B, g = _b.linearize_discretize_batch(np.asarray(x_bar, np.float64).reshape(1, 6),
                                            np.asarray(u_bar, np.float64).reshape(1, 2), Ts, p)
    return _np(A)[0], _np(B)[0], _np(g)[0]


def lateral_error(X, Y, Xref, Yref, phiref):
    """e_c = sin(phi_ref)(X - Xref) - cos(phi_ref)(Y - Yref) -- mpc_6stati.py:111-117 (HIP kernel)."""
    args = [np.asarray(v, np.float64) for v in (X, Y, Xref, Yref, phiref)]
    shape = np.broadcast(*args).shape
    flat = [np.broadcast_to(a, shape).reshape(-1) for a in args]
    out = _np(_b.lateral_error_batch(*flat)).reshape(shape)
    return out[()] if shape == () else out


def _is_psd(M):
    S = 0.5 * (M + M.T)
    w = np.linalg.eigvalsh(S)
    return w.min() >= -1e-12 * max(1.0, np.abs(w).max())


def mpc_step(
    x0,
    u_prev,
    path_ref,
    Ts=0.02,
    N=20,
    params=None,
    q_c=6.0,
    q_phi=0.5,
    q_vx=0.5,
    R=np.diag([0.02, 2.0]),
    Rd=np.diag([0.01, 5.0]),
    vref=None,
    u_bounds=((-1.0, 1.0), (-0.6, 0.6)),
    du_bounds=((-0.5, 0.5), (-0.3, 0.3)),
    x_lo=None,
    x_hi=None,
    solver="OSQP",
    verbose=False,
    **solver_settings,
):
    """One MPC step (mpc_6stati.py:120-275); see the module docstring for the contract."""
    p = dict(Params)
    if params is not None:
        p.update(params)
    x0 = np.asarray(x0).reshape(6).astype(np.float64)
    u_pr = np.asarray(u_prev).reshape(2).astype(np.float64)
    path_ref = np.asarray(path_ref)
    assert path_ref.shape[0] == N + 1 and path_ref.shape[1] == 3
    if vref is None:
        vref = np.full(N + 1, x0[3])
    elif np.isscalar(vref):
        vref = np.full(N + 1, float(vref))
    else:
        vref = np.asarray(vref).reshape(N + 1)
    R = np.asarray(R, dtype=np.float64)
    Rd = np.asarray(Rd, dtype=np.float64)
    if not (_is_psd_cached(R) and _is_psd_cached(Rd)):
        # cvxpy rejects a non-convex quad_form at prob.solve (inside the reference's try, :255-259)
        return u_pr, "Solver Error: DCPError", {}
    cfg = _cached_struct(
        "cfg", lambda: _b.config_struct(N=N, Ts=Ts, q_c=q_c, q_phi=q_phi, q_vx=q_vx, R=R, Rd=Rd, u_bounds=u_bounds,
                                        du_bounds=du_bounds, x_lo=x_lo, x_hi=x_hi, **solver_settings),
        N, Ts, q_c, q_phi, q_vx, R, Rd, u_bounds, du_bounds, x_lo, x_hi, tuple(sorted(solver_settings.items())))
    pk = _params_key(p)
    pst = (_cached_struct("params", lambda: _b.params_struct(p), key=pk) if pk is not None
           else _cached_struct("params", lambda: _b.params_struct(p), tuple(sorted(p.items()))))
    # one staged copy in: [x0 6 | u_prev 2 | path_ref 3(N+1) | vref N+1]; one copy out:
    # [u_cmd 2 | objective 1 | X_opt 6(N+1) | U_opt 2N | status, iters, polished (int32)]
    dev = _b.require_gpu()
    nin, nf = 8 + 4 * (N + 1), 3 + 6 * (N + 1) + 2 * N
    io = _CallIO.get(("mpc_step", N), dev, nin, nf, 3)
    a = io.a_in
    a[:6] = x0
    a[6:8] = u_pr
    a[8:8 + 3 * (N + 1)] = np.asarray(path_ref, np.float64).reshape(-1)
    a[8 + 3 * (N + 1):] = np.asarray(vref, np.float64).reshape(-1)
    io.send()
    # the step entry point on the staged buffers directly (batch.mpc_step_batch's launch for B = 1, without its
    # per-call tensor views and conversions)
    sb = int(_b._lib.lib().traj_mpc_sb_workspace_bytes(1, N)) if _b._general(cfg) else 0
    ws = _b.workspace(1, N, dev, sb, role="step")
    try:
        _b._lib.check(_b._lib.lib().traj_mpc_step_batch(C.byref(pst), C.byref(cfg), 1, *io.step_ptrs(N),
                                                        C.c_void_p(ws.data_ptr()), ws.numel() * 8,
                                                        C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                      "traj_mpc_step_batch")
    except BaseException:
        io.abort()
        raise
    h = io.receive()
    st = int(h[nf:].view(np.int32)[0])
    status = STATUS_STRINGS.get(st, "Solver Error: SolverError")
    if st == 6:
        return u_pr, status, {}
    if status not in ("optimal", "optimal_inaccurate"):
        return u_pr, status, {}
    u_cmd = h[0:2].copy()
    info = {
        "status": status,
        "objective": float(h[2]),
        "X_opt": h[3:3 + 6 * (N + 1)].reshape(6, N + 1).copy(),
        "U_opt": h[3 + 6 * (N + 1):nf].reshape(2, N).copy(),
        "path_ref": path_ref,
        "vref": vref,
    }
    return u_cmd, status, info


def mpc_step_batch(x0, u_prev, path_ref, vref=None, Ts=0.02, N=20, params=None, **kwargs):
    """Batched mpc_step: x0 [B,6], u_prev [B,2], path_ref [B,N+1,3], vref [B,N+1] / [N+1] / scalar / None.
    Returns a dict of torch.cuda tensors (see batch.mpc_step_batch)."""
    x0 = torch.as_tensor(x0, dtype=torch.float64)
    B = x0.reshape(-1, 6).shape[0]
    if vref is None:
        vref = x0.reshape(B, 6)[:, 3:4].expand(B, N + 1)
    elif np.isscalar(vref):
        vref = torch.full((B, N + 1), float(vref), dtype=torch.float64)
    else:
        vref = torch.as_tensor(vref, dtype=torch.float64)
        if vref.dim() == 1:
            vref = vref.reshape(1, N + 1).expand(B, N + 1)
    solver_keys = {k: kwargs.pop(k) for k in list(kwargs) if k not in (
        "q_c", "q_phi", "q_vx", "R", "Rd", "u_bounds", "du_bounds", "x_lo", "x_hi")}
    solver_keys.pop("solver", None)
    solver_keys.pop("verbose", None)
    cfg = _b.config_struct(N=N, Ts=Ts, **kwargs, **solver_keys)
    return _b.mpc_step_batch(x0, u_prev, path_ref, vref, cfg, params)
