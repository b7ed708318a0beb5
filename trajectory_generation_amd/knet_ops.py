"""The KalmanNet step's HIP ops registered with torch.library (``torch.ops.trajknet.*``).

  torch.ops.trajknet.prior(x_post, u, y, x_mean, x_std, y_mean, y_std, u_mean, u_std, params, limits, Ts)
      -> (m1x_prior [B,6], m1y [B,5], dy [B,5])          kalman_net.py:145-162 (traj_knet_prior_f32)
  torch.ops.trajknet.gru_gates(gi, gh, h) -> h_out       one torch.nn.GRU cell's gates (traj_knet_gru_gates_f32)
  torch.ops.trajknet.update(m1x_prior, KG, dy, innov_logit) -> x_post
                                                          kalman_net.py:169-178 (traj_knet_update_f32)
  torch.ops.trajknet.pack(weights, dims) -> packed        the fused kernels' packed weight copy (traj_knet_pack_f32)
  torch.ops.trajknet.step(y, u, x_post, h_q, h_sigma, h_s, packed, weights, dims, params, limits, Ts, norm)
      -> (x_post, h_q, h_sigma, h_s, KG)                  kalman_net.py:145-216, one whole eval-mode step as the
                                                          fused front -> fc2 -> back launches

Functional: no input is modified (the step's hidden states come back as new tensors).  Every op has a fake
(meta) kernel, so shapes propagate under FakeTensorMode / torch.compile tracing without a GPU; prior,
gru_gates and update carry autograd formulas (the reference's expressions, as knet.py's training path).
The real kernels need the HIP library and a GPU -- there is no CPU implementation.

``weights`` is the list ``step_weights(model)`` returns (traj_knet_net's pointer fields, in order),
``dims`` = [m, n, hidden, d_fc5, d_fc1, d_fc7, d_fc3, d_fc2h], ``params`` the traj_vehicle_params fields in
order (``params_list``), ``limits`` the 12 clamp limits (knet.LIMIT_KEYS order), ``norm`` = [x_mean, x_std,
y_mean, y_std] (+ [u_mean, u_std] when the controls are normalized).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import torch
from torch.library import custom_op, register_fake

from . import _lib
from .batch import REFERENCE_PARAMS

NET_PTRS = ("fc5_w", "fc5_b", "gru_q_wih", "gru_q_bih", "gru_q_whh", "gru_q_bhh", "gru_sigma_wih", "gru_sigma_bih",
            "gru_sigma_whh", "gru_sigma_bhh", "fc1_w", "fc1_b", "fc7_w", "fc7_b", "gru_s_wih", "gru_s_bih",
            "gru_s_whh", "gru_s_bhh", "fc3_w", "fc3_b", "fc4_w", "fc4_b", "innov_logit", "fc2a_w", "fc2a_b",
            "fc2b_w", "fc2b_b")
DIMS = ("m", "n", "hidden", "d_fc5", "d_fc1", "d_fc7", "d_fc3", "d_fc2h")
PARAM_KEYS = tuple(k for k, _ in _lib.VehicleParams._fields_)
LIMIT_KEYS = ("x_min", "x_max", "y_min", "y_max", "phi_min", "phi_max", "vx_min", "vx_max", "vy_min", "vy_max",
              "omega_min", "omega_max")


def params_list(params: dict | None = None) -> List[float]:
    """traj_vehicle_params fields in order (reference Params + overrides)."""
    p = dict(REFERENCE_PARAMS)
    p.update(params or {})
    return [float(p[k]) for k in PARAM_KEYS]


def limits_list(params: dict) -> List[float]:
    """The 12 clamp limits of vehicle_model.py (KeyError if one is missing, as the reference's p["phi_min"])."""
    return [float(params[k]) for k in LIMIT_KEYS]


def step_weights(model) -> List[torch.Tensor]:
    """The fused step's weight list of a built KalmanNetNN (traj_knet_net's pointer fields, in order)."""
    lin = {"fc5": model.FC5[0], "fc1": model.FC1[0], "fc7": model.FC7[0], "fc3": model.FC3[0], "fc4": model.FC4[0],
           "fc2a": model.FC2[0], "fc2b": model.FC2[2]}
    gru = {"gru_q": model.GRU_Q, "gru_sigma": model.GRU_Sigma, "gru_s": model.GRU_S}
    gk = {"wih": "weight_ih_l0", "bih": "bias_ih_l0", "whh": "weight_hh_l0", "bhh": "bias_hh_l0"}
    out = []
    for k in NET_PTRS:
        if k == "innov_logit":
            out.append(model.innov_logit.detach())
            continue
        base, part = k.rsplit("_", 1)
        if base in gru:
            out.append(getattr(gru[base], gk[part]).detach())
        else:
            out.append((lin[base].weight if part == "w" else lin[base].bias).detach())
    return out


def step_dims(model) -> List[int]:
    return [model.m, model.n, model.d_hidden_Q, model.d_output_FC5, model.d_output_FC1, model.d_output_FC7,
            model.d_output_FC3, model.d_hidden_FC2]


# ---------------------------------------------------------------- helpers

def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream(dev):
    return C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _params_struct(vals: Sequence[float]) -> _lib.VehicleParams:
    s = _lib.VehicleParams()
    for k, v in zip(PARAM_KEYS, vals):
        setattr(s, k, float(v))
    return s


def _limits_struct(vals: Sequence[float]) -> _lib.KnetLimits:
    s = _lib.KnetLimits()
    for k, v in zip(LIMIT_KEYS, vals):
        setattr(s, k, float(v))
    return s


def _net_struct(weights: Sequence[torch.Tensor], dims: Sequence[int]) -> _lib.KnetNet:
    if len(weights) != len(NET_PTRS) or len(dims) != len(DIMS):
        raise ValueError(f"trajknet: {len(NET_PTRS)} weights and {len(DIMS)} dims expected")
    w = _lib.KnetNet()
    for k, v in zip(DIMS, dims):
        setattr(w, k, int(v))
    for k, t in zip(NET_PTRS, weights):
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise ValueError(f"trajknet: {k} must be a contiguous float32 device tensor")
        setattr(w, k, t.data_ptr())
    return w


def _f32(t, B, c):
    return t.reshape(B, c).to(torch.float32).contiguous()


def _norm_args(norm: Sequence[torch.Tensor]):
    if len(norm) not in (4, 6):
        raise ValueError("trajknet: norm = [x_mean, x_std, y_mean, y_std] (+ [u_mean, u_std])")
    ts = [t.reshape(-1).to(torch.float32).contiguous() for t in norm]
    return ts + [None, None] if len(ts) == 4 else ts


# ---------------------------------------------------------------- prior

@custom_op("trajknet::prior", mutates_args=())
def prior(x_post: torch.Tensor, u: torch.Tensor, y: torch.Tensor, x_mean: torch.Tensor, x_std: torch.Tensor,
          y_mean: torch.Tensor, y_std: torch.Tensor, u_mean: Optional[torch.Tensor], u_std: Optional[torch.Tensor],
          params: List[float], limits: List[float], Ts: float) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    B = x_post.shape[0]
    dev = x_post.device
    xp, uu, yy = _f32(x_post, B, 6), _f32(u, B, 2), _f32(y, B, 5)
    norm = _norm_args([x_mean, x_std, y_mean, y_std] + ([u_mean, u_std] if u_mean is not None and u_std is not None
                                                         else []))
    out = [torch.empty((B, c), dtype=torch.float32, device=dev) for c in (6, 5, 5)]
    _lib.check(_lib.lib().traj_knet_prior_f32(
        C.byref(_params_struct(params)), C.byref(_limits_struct(limits)), float(Ts), B, _p(xp), _p(uu), _p(yy),
        *[_p(t) for t in norm], *[_p(t) for t in out], _stream(dev)), "trajknet::prior")
    return out[0], out[1], out[2]


@register_fake("trajknet::prior")
def _prior_fake(x_post, u, y, x_mean, x_std, y_mean, y_std, u_mean, u_std, params, limits, Ts):
    B = x_post.shape[0]
    return tuple(x_post.new_empty((B, c), dtype=torch.float32) for c in (6, 5, 5))


def _prior_setup(ctx, inputs, output):
    x_post, u, y, x_mean, x_std, y_mean, y_std, u_mean, u_std, params, limits, Ts = inputs
    ctx.save_for_backward(x_post, u, y, x_mean, x_std, y_mean, y_std)
    ctx.u_norm = (u_mean, u_std)
    ctx.params, ctx.limits, ctx.Ts = params, limits, Ts


def _prior_backward(ctx, g_prior, g_m1y, g_dy):
    from .knet import torch_prior
    x_post, u, y, x_mean, x_std, y_mean, y_std = ctx.saved_tensors
    p = dict(zip(PARAM_KEYS, ctx.params))
    p.update(zip(LIMIT_KEYS, ctx.limits))
    with torch.enable_grad():
        xp = x_post.detach().reshape(-1, 6).requires_grad_(True)
        outs = torch_prior(p, ctx.Ts, xp, u.reshape(-1, 2), y.reshape(-1, 5), x_mean, x_std, y_mean, y_std,
                           *ctx.u_norm)
        pairs = [(o, g) for o, g in zip(outs, (g_prior, g_m1y, g_dy)) if g is not None]
        gx, = torch.autograd.grad([o for o, _ in pairs], [xp], [g for _, g in pairs])
    return (gx.reshape(x_post.shape),) + (None,) * 11


prior.register_autograd(_prior_backward, setup_context=_prior_setup)


# ---------------------------------------------------------------- GRU gates

@custom_op("trajknet::gru_gates", mutates_args=())
def gru_gates(gi: torch.Tensor, gh: torch.Tensor, h: torch.Tensor) -> torch.Tensor:
    B, H = h.shape
    if gi.shape != (B, 3 * H) or gh.shape != (B, 3 * H):
        raise ValueError("trajknet::gru_gates: gi, gh [B, 3H], h [B, H]")
    gi, gh, h = (t.to(torch.float32).contiguous() for t in (gi, gh, h))
    out = torch.empty_like(h)
    _lib.check(_lib.lib().traj_knet_gru_gates_f32(B, H, _p(gi), _p(gh), _p(h), _p(out), _stream(h.device)),
               "trajknet::gru_gates")
    return out


@register_fake("trajknet::gru_gates")
def _gru_gates_fake(gi, gh, h):
    return torch.empty_like(h, dtype=torch.float32)


def _gates_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _gates_backward(ctx, g):
    from .knet import torch_gru_gates
    gi, gh, h = ctx.saved_tensors
    with torch.enable_grad():
        a, b, c = (t.detach().requires_grad_(True) for t in (gi, gh, h))
        return torch.autograd.grad(torch_gru_gates(a, b, c), [a, b, c], [g])


gru_gates.register_autograd(_gates_backward, setup_context=_gates_setup)


# ---------------------------------------------------------------- posterior update

@custom_op("trajknet::update", mutates_args=())
def update(m1x_prior: torch.Tensor, KG: torch.Tensor, dy: torch.Tensor, innov_logit: torch.Tensor) -> torch.Tensor:
    B, m = m1x_prior.shape
    n = dy.shape[1]
    if KG.numel() != B * m * n:
        raise ValueError("trajknet::update: KG must hold B * m * n values")
    pr, kg, d, lg = (t.to(torch.float32).contiguous() for t in (m1x_prior, KG, dy, innov_logit))
    post = torch.empty((B, m), dtype=torch.float32, device=m1x_prior.device)
    _lib.check(_lib.lib().traj_knet_update_f32(B, _p(pr), _p(kg), _p(d), _p(lg), _p(post), _stream(pr.device)),
               "trajknet::update")
    return post


@register_fake("trajknet::update")
def _update_fake(m1x_prior, KG, dy, innov_logit):
    return m1x_prior.new_empty(m1x_prior.shape, dtype=torch.float32)


def _update_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _update_backward(ctx, g):
    prior_, KG, dy, logit = ctx.saved_tensors
    with torch.enable_grad():
        ts = [t.detach().requires_grad_(True) for t in (prior_, KG, dy, logit)]
        B, m = prior_.shape
        n = dy.shape[1]
        post = ts[0] + (torch.sigmoid(ts[3]) * torch.bmm(ts[1].reshape(B, m, n), ts[2].reshape(B, n, 1))).reshape(B, m)
        return torch.autograd.grad(post, ts, [g])


update.register_autograd(_update_backward, setup_context=_update_setup)


# ---------------------------------------------------------------- fused step (inference)

@custom_op("trajknet::pack", mutates_args=())
def pack(weights: List[torch.Tensor], dims: List[int]) -> torch.Tensor:
    net = _net_struct(weights, dims)
    L = _lib.lib()
    nbytes = L.traj_knet_packed_bytes(C.byref(net))
    if nbytes == 0:
        raise NotImplementedError("trajknet::pack: unsupported network shape")
    dev = weights[0].device
    out = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    _lib.check(L.traj_knet_pack_f32(C.byref(net), _p(out), nbytes, _stream(dev)), "trajknet::pack")
    return out


@register_fake("trajknet::pack")
def _pack_fake(weights, dims):
    # the packed size depends only on the shapes: traj_knet_packed_bytes of a pointer-free net (host arithmetic)
    net = _lib.KnetNet()
    for k, v in zip(DIMS, dims):
        setattr(net, k, int(v))
    for k in NET_PTRS:   # (only checked for presence, never dereferenced, by the size computation)
        setattr(net, k, 16)
    nbytes = _lib.lib().traj_knet_packed_bytes(C.byref(net))
    if nbytes == 0:
        raise NotImplementedError("trajknet::pack: unsupported network shape")
    return weights[0].new_empty((nbytes // 4,), dtype=torch.float32)


@custom_op("trajknet::step", mutates_args=())
def step(y: torch.Tensor, u: torch.Tensor, x_post: torch.Tensor, h_q: torch.Tensor, h_sigma: torch.Tensor,
         h_s: torch.Tensor, packed: torch.Tensor, weights: List[torch.Tensor], dims: List[int], params: List[float],
         limits: List[float], Ts: float, norm: List[torch.Tensor]
         ) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    m, n, H = dims[0], dims[1], dims[2]
    B = x_post.shape[0]
    dev = x_post.device
    net = _net_struct(weights, dims)
    L = _lib.lib()
    st = _stream(dev)
    yy, uu, post = _f32(y, B, n), _f32(u, B, 2), _f32(x_post, B, m)
    hq, hsig, hs = (_f32(t, B, H).clone() for t in (h_q, h_sigma, h_s))
    nrm = _norm_args(norm)
    f = lambda *sh: torch.empty(sh, dtype=torch.float32, device=dev)   # noqa: E731
    prior_, dy, x2, KG, out = f(B, m), f(B, n), f(B, 2 * H), f(B, n * m), f(B, m)
    ws = f(L.traj_knet_fc2_workspace_bytes(C.byref(net), B) // 4)
    pk = packed.contiguous()
    _lib.check(L.traj_knet_front_f32(C.byref(_params_struct(params)), C.byref(_limits_struct(limits)), float(Ts),
                                     C.byref(net), _p(pk), B, _p(post), _p(uu), 2, 1, _p(yy), n, 1,
                                     *[_p(t) for t in nrm], _p(hq), _p(hsig), _p(hs), _p(prior_), _p(dy), _p(x2), st),
               "trajknet::step (front)")
    _lib.check(L.traj_knet_fc2_f32(C.byref(net), B, _p(x2), _p(ws), ws.numel() * 4, st), "trajknet::step (fc2)")
    _lib.check(L.traj_knet_back_f32(C.byref(net), _p(pk), B, _p(x2), _p(ws), _p(prior_), _p(dy), _p(hsig), _p(out),
                                    None, 0, 0, _p(KG), st), "trajknet::step (back)")
    return out, hq, hsig, hs, KG


@register_fake("trajknet::step")
def _step_fake(y, u, x_post, h_q, h_sigma, h_s, packed, weights, dims, params, limits, Ts, norm):
    m, n, H = dims[0], dims[1], dims[2]
    B = x_post.shape[0]
    e = lambda c: x_post.new_empty((B, c), dtype=torch.float32)   # noqa: E731
    return e(m), e(H), e(H), e(H), e(n * m)
