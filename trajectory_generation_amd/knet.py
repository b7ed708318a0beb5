"""KalmanNet inference on MI355X: drop-in for KalmanNet/kalman_net.py (KalmanNetNN) and
KalmanNet/vehicle_model.py (VehicleModel), float32 like the reference.

Same class names, constructor/NNBuild arguments, attributes (``batch_size``, ``m1x_posterior``,
``h_Q`` / ``h_Sigma`` / ``h_S``, ``KGain``, ``f`` / ``h``) and ``state_dict`` keys as the reference, so
its checkpoints load unchanged.  What runs on the device per step (kalman_net.py:169-216):

* ``traj_knet_prior_f32``   (HIP) denormalize, vehicle f (clamped Euler step), h, renormalize, and the
  innovation y - m1y: kalman_net.py:145-162 in one kernel;
* the gain network's dense layers as library GEMMs (``torch.addmm`` -> hipBLASLt), ReLU in place;
* ``traj_knet_gru_gates_f32`` (HIP) the three GRU cells' gate arithmetic after their two GEMMs;
* ``traj_knet_update_f32`` (HIP) x_post = x_prior + sigmoid(innov_logit) * KG dy (:169-178).

``KNetSequenceRunner`` captures one whole step in a HIP graph and replays it T times; its fused mode
(the throughput path) runs a step as ``traj_knet_front_f32`` (prior + FC5 + the three GRU cells + FC1/FC7
for four sequences per workgroup), ``traj_knet_fc2_f32`` (FC2 on the bf16 matrix cores with every
f32 operand carried as three bf16 terms -- f32-accurate sums -- its [B, 10240] hidden activation kept
on chip) and ``traj_knet_back_f32`` (FC3 + FC4 + posterior update), with back(t)
and front(t + 1) fused into one launch (``traj_knet_back_front_f32``), and captures all T steps in one
graph.
There is no CPU path: the ops raise without the HIP library or a GPU.

Training (``knet_train.py``): with autograd on, the three HIP ops run inside
``torch.autograd.Function`` s whose backward re-evaluates the same step in torch ops on the device
and differentiates it -- the expressions of vehicle_model.py / kalman_net.py that the reference's
autograd differentiates (clamp, max and atan2 subgradients included); the GEMMs are torch's.
"""
from __future__ import annotations

import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from .batch import REFERENCE_PARAMS, params_struct, require_gpu

Params = dict(REFERENCE_PARAMS)

LIMIT_KEYS = ("x_min", "x_max", "y_min", "y_max", "phi_min", "phi_max", "vx_min", "vx_max", "vy_min", "vy_max",
              "omega_min", "omega_max")


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def limits_struct(params: dict) -> _lib.KnetLimits:
    missing = [k for k in LIMIT_KEYS if k not in params]
    if missing:
        # vehicle_model.py:54 reads p["phi_min"] etc.; the reference raises KeyError without them
        raise KeyError(missing[0])
    s = _lib.KnetLimits()
    for k in LIMIT_KEYS:
        setattr(s, k, float(params[k]))
    return s


def knet_prior(params: dict, Ts: float, x_post, u, x_mean, x_std, y_mean, y_std, y=None, u_mean=None, u_std=None):
    """kalman_net.py:145-162 for B sequences: returns (m1x_prior [B,6], m1y [B,5], dy [B,5] or None)."""
    dev = x_post.device
    B = x_post.shape[0]
    xp = x_post.reshape(B, 6).contiguous()
    uu = u.reshape(B, 2).contiguous()
    yy = None if y is None else y.reshape(B, 5).contiguous()
    prior = torch.empty((B, 6), dtype=torch.float32, device=dev)
    m1y = torch.empty((B, 5), dtype=torch.float32, device=dev)
    dy = None if y is None else torch.empty((B, 5), dtype=torch.float32, device=dev)
    # bound to locals: a temporary's storage would go back to the allocator before the launch
    norm = [None if t is None else t.reshape(-1).contiguous() for t in (x_mean, x_std, y_mean, y_std, u_mean, u_std)]
    _lib.check(_lib.lib().traj_knet_prior_f32(
        C.byref(params_struct(params)), C.byref(limits_struct(params)), float(Ts), B, _p(xp), _p(uu), _p(yy),
        *[_p(t) for t in norm], _p(prior), _p(m1y), _p(dy), _stream()), "traj_knet_prior_f32")
    return prior, m1y, dy


def _gru_gates(gi, gh, h):
    out = torch.empty_like(h)
    B, H = h.shape
    gi, gh, h = gi.contiguous(), gh.contiguous(), h.contiguous()
    _lib.check(_lib.lib().traj_knet_gru_gates_f32(B, H, _p(gi), _p(gh), _p(h), _p(out), _stream()),
               "traj_knet_gru_gates_f32")
    return out


def gru_cell(x, h, gru: nn.GRU):
    """One step of a 1-layer torch.nn.GRU: two GEMMs + the fused gate kernel. x [B,in], h [B,H]."""
    gi = torch.addmm(gru.bias_ih_l0, x, gru.weight_ih_l0.t())
    gh = torch.addmm(gru.bias_hh_l0, h, gru.weight_hh_l0.t())
    if torch.is_grad_enabled() and (gi.requires_grad or gh.requires_grad or h.requires_grad):
        return _GruGatesFn.apply(gi, gh, h)
    return _gru_gates(gi, gh, h)


# ---------------------------------------------------------------- autograd (training, f4)

def torch_prior(params: dict, Ts: float, x_post, u, y, x_mean, x_std, y_mean, y_std, u_mean=None, u_std=None):
    """kalman_net.py:145-162 with vehicle_model.py:19-153 in torch ops on [B,6] / [B,2] / [B,5] tensors:
    the expressions whose autograd the reference runs, evaluated by knet_prior's backward."""
    p = params
    xs, xm = x_std.reshape(1, 6), x_mean.reshape(1, 6)
    x = x_post * xs + xm                                                   # _denorm_x
    uu = u if (u_mean is None or u_std is None) else u * u_std.reshape(1, 2) + u_mean.reshape(1, 2)
    phi = torch.clamp(x[:, 2], p["phi_min"], p["phi_max"])                # pt_f_cont (:45-79)
    vx = torch.clamp(x[:, 3], p["vx_min"], p["vx_max"])
    vy = torch.clamp(x[:, 4], p["vy_min"], p["vy_max"])
    omega = torch.clamp(x[:, 5], p["omega_min"], p["omega_max"])
    d, delta = uu[:, 0], uu[:, 1]
    vx_eff = torch.max(torch.abs(vx), torch.tensor(p["vx_zero"], device=vx.device))   # pt_tire_forces (:19-42)
    alpha_f = -torch.atan2(omega * p["lf"] + vy, vx_eff) + delta
    alpha_r = torch.atan2(omega * p["lr"] - vy, vx_eff)
    alpha_f = torch.clamp(alpha_f, -p["maxAlpha"], p["maxAlpha"])
    Fy_f = p["Df"] * torch.sin(p["Cf"] * torch.atan(p["Bf"] * alpha_f))
    Fy_r = p["Dr"] * torch.sin(p["Cr"] * torch.atan(p["Br"] * alpha_r))
    Frx = (p["Cm1"] - p["Cm2"] * vx_eff) * d - p["Cr0"] - p["Cr2"] * (vx_eff ** 2)
    m, Iz, lf, lr = p["m"], p["Iz"], p["lf"], p["lr"]
    xdot = torch.stack([vx * torch.cos(phi) - vy * torch.sin(phi), vx * torch.sin(phi) + vy * torch.cos(phi), omega,
                        (Frx - Fy_f * torch.sin(delta) + m * vy * omega) / m,
                        (Fy_r + Fy_f * torch.cos(delta) - m * vx * omega) / m,
                        (Fy_f * lf * torch.cos(delta) - Fy_r * lr) / Iz], dim=1)
    xn = x + Ts * xdot                                                      # f (:109-134)
    lim = [("x_min", "x_max"), ("y_min", "y_max"), ("phi_min", "phi_max"), ("vx_min", "vx_max"),
           ("vy_min", "vy_max"), ("omega_min", "omega_max")]
    xn = torch.stack([torch.clamp(xn[:, i], p[a], p[b]) for i, (a, b) in enumerate(lim)], dim=1)
    prior = (xn - xm) / xs                                                  # _renorm_x
    m1y = (xn[:, [0, 1, 3, 4, 5]] - y_mean.reshape(1, 5)) / y_std.reshape(1, 5)   # h, _renorm_y
    return prior, m1y, y - m1y


class _KnetPriorFn(torch.autograd.Function):
    """knet_prior (HIP) forward; backward through torch_prior w.r.t. x_post."""

    @staticmethod
    def forward(ctx, x_post, u, y, params, Ts, norm):
        prior, m1y, dy = knet_prior(params, Ts, x_post, u, *norm[:4], y=y, u_mean=norm[4], u_std=norm[5])
        ctx.save_for_backward(x_post, u, y)
        ctx.params, ctx.Ts, ctx.norm = params, Ts, norm
        return prior, m1y, dy

    @staticmethod
    def backward(ctx, g_prior, g_m1y, g_dy):
        x_post, u, y = ctx.saved_tensors
        with torch.enable_grad():
            xp = x_post.detach().reshape(-1, 6).requires_grad_(True)
            outs = torch_prior(ctx.params, ctx.Ts, xp, u.reshape(-1, 2), y.reshape(-1, 5), *ctx.norm)
            pairs = [(o, g) for o, g in zip(outs, (g_prior, g_m1y, g_dy)) if g is not None]
            gx, = torch.autograd.grad([o for o, _ in pairs], [xp], [g for _, g in pairs])
        return gx.reshape(x_post.shape), None, None, None, None, None


def torch_gru_gates(gi, gh, h):
    """torch.nn.GRU's gate arithmetic (r, z, n order) on the two GEMM outputs."""
    H = h.shape[1]
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return (1.0 - z) * n + z * h


class _GruGatesFn(torch.autograd.Function):
    """traj_knet_gru_gates_f32 forward; backward through torch_gru_gates."""

    @staticmethod
    def forward(ctx, gi, gh, h):
        ctx.save_for_backward(gi, gh, h)
        return _gru_gates(gi, gh, h)

    @staticmethod
    def backward(ctx, g):
        gi, gh, h = ctx.saved_tensors
        with torch.enable_grad():
            a, b, c = (t.detach().requires_grad_(True) for t in (gi, gh, h))
            return torch.autograd.grad(torch_gru_gates(a, b, c), [a, b, c], [g])


class _UpdateFn(torch.autograd.Function):
    """traj_knet_update_f32 forward: x_post = x_prior + sigmoid(innov_logit) KG dy (kalman_net.py:169-178)."""

    @staticmethod
    def forward(ctx, prior, KG, dy, logit):
        B, m = prior.shape
        post = torch.empty((B, m), dtype=torch.float32, device=prior.device)
        prior_c, KG_c, dy_c, lg = prior.contiguous(), KG.contiguous(), dy.contiguous(), logit.detach().contiguous()
        _lib.check(_lib.lib().traj_knet_update_f32(B, _p(prior_c), _p(KG_c), _p(dy_c), _p(lg), _p(post), _stream()),
                   "traj_knet_update_f32")
        ctx.save_for_backward(prior, KG, dy, logit)
        return post

    @staticmethod
    def backward(ctx, g):
        prior, KG, dy, logit = ctx.saved_tensors
        with torch.enable_grad():
            ts = [t.detach().requires_grad_(True) for t in (prior, KG, dy, logit)]
            B, m = prior.shape
            n = dy.shape[1]
            post = ts[0] + (torch.sigmoid(ts[3]) * torch.bmm(ts[1].reshape(B, m, n), ts[2].reshape(B, n, 1))).reshape(B, m)
            return torch.autograd.grad(post, ts, [g])


def _linear(x, lin: nn.Linear, relu: bool):
    y = torch.addmm(lin.bias, x, lin.weight.t())
    return F.relu_(y) if relu else y


class VehicleModel:
    """vehicle_model.py:81-153.  ``Params`` must carry the 12 clamp limits (``LIMIT_KEYS``)."""

    def __init__(self, Ts, T_train, T_test, m1x_0_real, prior_Q=None, prior_Sigma=None, prior_S=None):
        self.m, self.n, self.d = 6, 5, 2
        self.Ts = Ts
        self.Params = dict(Params)
        self.T, self.T_test = T_train, T_test
        self.m1x_0 = m1x_0_real
        self.prior_Q, self.prior_Sigma, self.prior_S = prior_Q, prior_Sigma, prior_S

    def f(self, x_batch_in, u_batch_in):
        """x [B,6,1], u [B,2,1] -> clamped Euler step [B,6,1] (vehicle_model.py:109-134)."""
        dev = x_batch_in.device
        one6 = torch.ones(6, dtype=torch.float32, device=dev)
        one5 = torch.ones(5, dtype=torch.float32, device=dev)
        prior, _, _ = knet_prior(self.Params, self.Ts, x_batch_in.float(), u_batch_in.float(),
                                 torch.zeros_like(one6), one6, torch.zeros_like(one5), one5)
        return prior.unsqueeze(2)

    def h(self, x_batch_in):
        """rows X, Y, vx, vy, omega (vehicle_model.py:136-153)."""
        idx = torch.tensor([0, 1, 3, 4, 5], device=x_batch_in.device)
        return torch.index_select(x_batch_in, 1, idx)


class KalmanNetNN(nn.Module):
    """kalman_net.py:5-223 with the step fused on the device (see the module docstring)."""

    def __init__(self, device=None):
        super().__init__()
        self.device = require_gpu(device)
        self.has_norm_params_xy = False
        self.has_norm_params_u = False
        self.u_mean = self.u_std = None

    def set_normalization(self, x_mean, x_std, y_mean, y_std, u_mean=None, u_std=None):
        self.x_mean = x_mean.to(self.device, torch.float32)
        self.x_std = x_std.to(self.device, torch.float32)
        self.y_mean = y_mean.to(self.device, torch.float32)
        self.y_std = y_std.to(self.device, torch.float32)
        self.has_norm_params_xy = True
        if (u_mean is not None) and (u_std is not None):
            self.u_mean = u_mean.to(self.device, torch.float32)
            self.u_std = u_std.to(self.device, torch.float32)
            self.has_norm_params_u = True
        else:
            self.u_mean = self.u_std = None
            self.has_norm_params_u = False

    def NNBuild(self, SysModel, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128):
        """kalman_net.py:26-113: the same modules, shapes and names (state_dict compatible)."""
        self.innov_logit = nn.Parameter(torch.tensor(0.0))
        self.sys = SysModel
        self.f = SysModel.f
        self.h = SysModel.h
        self.m = SysModel.m
        self.n = SysModel.n
        self.seq_len_input = 1
        self.batch_size = 0
        m, n, H = self.m, self.n, hidden_dim_gru
        self.d_input_FC5, self.d_output_FC5 = m, m * in_mult_KNet
        self.FC5 = nn.Sequential(nn.Linear(m, m * in_mult_KNet), nn.ReLU(), nn.Dropout(p=0.05))
        self.d_input_Q, self.d_hidden_Q = self.d_output_FC5, H
        self.GRU_Q = nn.GRU(self.d_input_Q, H)
        self.d_input_Sigma, self.d_hidden_Sigma = H, H
        self.GRU_Sigma = nn.GRU(H, H)
        self.d_input_FC1, self.d_output_FC1 = H, n * n
        self.FC1 = nn.Sequential(nn.Linear(H, n * n), nn.ReLU(), nn.Dropout(p=0.05))
        self.d_input_FC7, self.d_output_FC7 = n, n
        self.FC7 = nn.Sequential(nn.Linear(n, n), nn.ReLU(), nn.Dropout(p=0.05))
        self.d_input_S, self.d_hidden_S = n * n + n, H
        self.GRU_S = nn.GRU(self.d_input_S, H)
        self.d_input_FC2 = 2 * H
        self.d_output_FC2 = n * m
        self.d_hidden_FC2 = self.d_input_FC2 * out_mult_KNet
        self.FC2 = nn.Sequential(nn.Linear(self.d_input_FC2, self.d_hidden_FC2), nn.ReLU(),
                                 nn.Linear(self.d_hidden_FC2, self.d_output_FC2), nn.Dropout(p=0.1))
        self.d_input_FC3, self.d_output_FC3 = H + n * m, m * m
        self.FC3 = nn.Sequential(nn.Linear(self.d_input_FC3, m * m), nn.ReLU(), nn.Dropout(p=0.05))
        self.d_input_FC4, self.d_output_FC4 = H + m * m, H
        self.FC4 = nn.Sequential(nn.Linear(self.d_input_FC4, H), nn.ReLU(), nn.Dropout(p=0.05))
        self.to(self.device)

    # ---------- normalization bridge (kalman_net.py:119-143) ----------
    def _denorm_x(self, x_norm):
        return x_norm * self.x_std + self.x_mean if self.has_norm_params_xy else x_norm

    def _renorm_x(self, x_real):
        return (x_real - self.x_mean) / self.x_std if self.has_norm_params_xy else x_real

    def _denorm_y(self, y_norm):
        return y_norm * self.y_std + self.y_mean if self.has_norm_params_xy else y_norm

    def _renorm_y(self, y_real):
        return (y_real - self.y_mean) / self.y_std if self.has_norm_params_xy else y_real

    def _denorm_u(self, u_in):
        return u_in * self.u_std + self.u_mean if self.has_norm_params_u else u_in

    def _norm_tensors(self):
        if self.has_norm_params_xy:
            return self.x_mean, self.x_std, self.y_mean, self.y_std
        dev = self.device
        return (torch.zeros(6, device=dev), torch.ones(6, device=dev), torch.zeros(5, device=dev),
                torch.ones(5, device=dev))

    def InitSequence(self, M1_0_norm, T):
        self.T = T
        self.m1x_posterior = M1_0_norm.to(self.device, torch.float32)

    def init_hidden_KNet(self):
        B, dev = self.batch_size, self.device
        self.h_S = torch.zeros((self.seq_len_input, B, self.d_hidden_S), device=dev)
        self.h_Sigma = torch.zeros((self.seq_len_input, B, self.d_hidden_Sigma), device=dev)
        self.h_Q = torch.zeros((self.seq_len_input, B, self.d_hidden_Q), device=dev)

    # ---------- one step ----------
    def step_prior(self, u, y=None):
        xm, xs, ym, ys = self._norm_tensors()
        if y is not None and torch.is_grad_enabled() and self.m1x_posterior.requires_grad:
            B = self.m1x_posterior.shape[0]
            prior, m1y, dy = _KnetPriorFn.apply(self.m1x_posterior.reshape(B, 6), u.reshape(B, 2).contiguous(),
                                                y.reshape(B, 5).contiguous(), self.sys.Params, self.sys.Ts,
                                                (xm, xs, ym, ys, self.u_mean, self.u_std))
        else:
            prior, m1y, dy = knet_prior(self.sys.Params, self.sys.Ts, self.m1x_posterior, u, xm, xs, ym, ys, y=y,
                                        u_mean=self.u_mean, u_std=self.u_std)
        self.m1x_prior = prior.unsqueeze(2)
        self.m1y = m1y.unsqueeze(2)
        return dy

    def KGain_step(self, obs_innov_diff, m1x_prior):
        """kalman_net.py:180-212: x [B,n] innovation, [B,m] prior -> FC2 output [B, n*m]."""
        drop = self.training
        def dp(x, mod):   # noqa: E306  (Dropout modules: identity in eval mode)
            return mod(x) if drop else x
        B = m1x_prior.shape[0]
        out_FC5 = dp(_linear(m1x_prior, self.FC5[0], True), self.FC5[2])
        h_Q = gru_cell(out_FC5, self.h_Q.reshape(B, -1), self.GRU_Q)
        out_Sigma = gru_cell(h_Q, self.h_Sigma.reshape(B, -1), self.GRU_Sigma)
        out_FC1 = dp(_linear(out_Sigma, self.FC1[0], True), self.FC1[2])
        out_FC7 = dp(_linear(obs_innov_diff, self.FC7[0], True), self.FC7[2])
        h_S = gru_cell(torch.cat((out_FC1, out_FC7), 1), self.h_S.reshape(B, -1), self.GRU_S)
        hid = _linear(torch.cat((out_Sigma, h_S), 1), self.FC2[0], True)
        out_FC2 = dp(_linear(hid, self.FC2[2], False), self.FC2[3])
        out_FC3 = dp(_linear(torch.cat((h_S, out_FC2), 1), self.FC3[0], True), self.FC3[2])
        out_FC4 = dp(_linear(torch.cat((out_Sigma, out_FC3), 1), self.FC4[0], True), self.FC4[2])
        self.h_Q = h_Q.unsqueeze(0)
        self.h_S = h_S.unsqueeze(0)
        self.h_Sigma = out_FC4.unsqueeze(0)
        return out_FC2

    def KNet_step(self, y, u):
        B = y.shape[0]
        dy = self.step_prior(u, y=y)
        KG = self.KGain_step(dy, self.m1x_prior.reshape(B, self.m))
        self.KGain = KG.reshape(self.batch_size, self.m, self.n)
        prior = self.m1x_prior.reshape(B, self.m)
        if torch.is_grad_enabled() and (prior.requires_grad or KG.requires_grad or self.innov_logit.requires_grad):
            post = _UpdateFn.apply(prior, KG, dy, self.innov_logit)
        else:
            post = torch.empty((B, self.m), dtype=torch.float32, device=self.device)
            prior, KGc = prior.contiguous(), KG.contiguous()
            _lib.check(_lib.lib().traj_knet_update_f32(B, _p(prior), _p(KGc), _p(dy), _p(self.innov_logit.detach()),
                                                       _p(post), _stream()), "traj_knet_update_f32")
        self.m1x_posterior = post.unsqueeze(2)
        return self.m1x_posterior

    def forward(self, y, u):
        """y [B,n,1] normalized, u [B,m_u,1] -> normalized posterior [B,m,1] (kalman_net.py:214-216)."""
        return self.KNet_step(y.to(self.device, torch.float32), u.to(self.device, torch.float32))


def net_struct(model: "KalmanNetNN") -> _lib.KnetNet:
    """traj_knet_net of a built KalmanNetNN (weights must stay alive and in place while it is used;
    the fused kernels read a packed copy of the matrices, made by traj_knet_pack_f32, and the biases here)."""
    w = _lib.KnetNet()
    w.m, w.n, w.hidden = model.m, model.n, model.d_hidden_Q
    w.d_fc5, w.d_fc1, w.d_fc7, w.d_fc3 = model.d_output_FC5, model.d_output_FC1, model.d_output_FC7, model.d_output_FC3
    mods = {"fc5": model.FC5[0], "fc1": model.FC1[0], "fc7": model.FC7[0], "fc3": model.FC3[0], "fc4": model.FC4[0]}
    for k, lin in mods.items():
        for t in (lin.weight, lin.bias):
            if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"{k}: fused KNet step needs contiguous float32 device weights")
        setattr(w, k + "_w", lin.weight.data_ptr())
        setattr(w, k + "_b", lin.bias.data_ptr())
    for k, g in {"gru_q": model.GRU_Q, "gru_sigma": model.GRU_Sigma, "gru_s": model.GRU_S}.items():
        for a in ("wih", "bih", "whh", "bhh"):
            t = getattr(g, {"wih": "weight_ih_l0", "bih": "bias_ih_l0", "whh": "weight_hh_l0", "bhh": "bias_hh_l0"}[a])
            if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"{k}: fused KNet step needs contiguous float32 device weights")
            setattr(w, f"{k}_{a}", t.data_ptr())
    w.innov_logit = model.innov_logit.data_ptr()
    w.d_fc2h = model.d_hidden_FC2
    for k, lin in {"fc2a": model.FC2[0], "fc2b": model.FC2[2]}.items():
        for t in (lin.weight, lin.bias):
            if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
                raise ValueError(f"{k}: fused KNet step needs contiguous float32 device weights")
        setattr(w, k + "_w", lin.weight.data_ptr())
        setattr(w, k + "_b", lin.bias.data_ptr())
    return w


class KNetSequenceRunner:
    """T steps of a KalmanNetNN (eval mode) for B sequences, one step captured in a HIP graph.

    Mirrors the inference loop of training_prediction.py:118-137 / test_vehicle.py:123-145:
    init_hidden_KNet, InitSequence(m1x0), then forward(y[:, :, t], u[:, :, t]) for t < T."""

    def __init__(self, model: KalmanNetNN, B: int, groups: int = 1, merge: bool = True):
        """groups: the fused mode's sequences split into that many independent launch chains (graph
        branches), so one group's latency-bound GRU kernels overlap another's FC2 on the matrix cores.
        merge: back(t) and front(t + 1) as one launch (traj_knet_back_front_f32); False keeps them apart
        (bit-identical results; for tests)."""
        self.model, self.B, self.groups, self.merge = model, B, groups, merge
        dev = model.device
        self.y = torch.zeros((B, model.n, 1), device=dev)
        self.u = torch.zeros((B, 2, 1), device=dev)
        self.graph = None

    def _init_state(self, m1x0):
        md = self.model
        md.batch_size = self.B
        md.init_hidden_KNet()
        md.InitSequence(m1x0, 0)

    # ---------- fused mode: three launches per step, all T steps in one graph ----------
    def _fused_steps(self, T, steps, g):
        """Enqueue `steps` fused steps of row group g (rows r0:r1) on the current stream."""
        md, S = self.model, self.fs
        L = _lib.lib()
        xm, xs, ym, ys = S["norm"]
        n, m, H = md.n, md.m, md.d_hidden_Q
        r0, r1 = S["rows"][g]
        Bg, ws = r1 - r0, S["ws"][g]
        row = lambda key, width: C.c_void_p(S[key].data_ptr() + 4 * r0 * width)   # noqa: E731
        net, pk = C.byref(S["net"]), _p(S["pk"])
        ucol = lambda t: C.c_void_p(S["u"].data_ptr() + 4 * (r0 * 2 * T + t))   # noqa: E731
        ycol = lambda t: C.c_void_p(S["y"].data_ptr() + 4 * (r0 * n * T + t))   # noqa: E731
        ocol = lambda t: C.c_void_p(S["out"].data_ptr() + 4 * (r0 * m * T + t))   # noqa: E731
        norm = [_p(xm), _p(xs), _p(ym), _p(ys), _p(S["um"]), _p(S["us"])]
        # step t = fc2(t), then back(t) fused with front(t + 1): two launches per step after the first
        for t in range(steps):
            if t == 0:
                _lib.check(L.traj_knet_front_f32(
                    C.byref(S["p"]), C.byref(S["lim"]), float(md.sys.Ts), net, pk, Bg, row("post", m),
                    ucol(0), 2 * T, T, ycol(0), n * T, T, *norm, row("hQ", H), row("hSig", H), row("hS", H),
                    row("prior", m), row("dy", n), row("x2", 2 * H), _stream()), "traj_knet_front_f32")
            _lib.check(L.traj_knet_fc2_f32(net, Bg, row("x2", 2 * H), _p(ws), ws.numel() * 4, _stream()),
                       "traj_knet_fc2_f32")
            if t + 1 < steps and self.merge:
                _lib.check(L.traj_knet_back_front_f32(
                    C.byref(S["p"]), C.byref(S["lim"]), float(md.sys.Ts), net, pk, Bg, _p(ws), ocol(t), m * T, T,
                    ucol(t + 1), 2 * T, T, ycol(t + 1), n * T, T, *norm, row("hQ", H), row("hSig", H), row("hS", H),
                    row("post", m), row("prior", m), row("dy", n), row("x2", 2 * H), _stream()),
                    "traj_knet_back_front_f32")
            else:
                _lib.check(L.traj_knet_back_f32(
                    net, pk, Bg, row("x2", 2 * H), _p(ws), row("prior", m), row("dy", n), row("hSig", H),
                    row("post", m), ocol(t), m * T, T, None, _stream()), "traj_knet_back_f32")
                if t + 1 < steps:
                    _lib.check(L.traj_knet_front_f32(
                        C.byref(S["p"]), C.byref(S["lim"]), float(md.sys.Ts), net, pk, Bg, row("post", m),
                        ucol(t + 1), 2 * T, T, ycol(t + 1), n * T, T, *norm, row("hQ", H), row("hSig", H),
                        row("hS", H), row("prior", m), row("dy", n), row("x2", 2 * H), _stream()),
                        "traj_knet_front_f32")

    def _enqueue_all(self, T, steps):
        """All row groups' steps; groups > 1 run as independent chains on side streams (graph branches)."""
        S = self.fs
        if len(S["rows"]) == 1:
            self._fused_steps(T, steps, 0)
            return
        main = torch.cuda.current_stream()
        for g, st in enumerate(S["streams"]):
            st.wait_stream(main)
            with torch.cuda.stream(st):
                self._fused_steps(T, steps, g)
        for st in S["streams"]:
            main.wait_stream(st)

    def _run_fused(self, y_seq, u_seq, m1x0, use_graph):
        md, B = self.model, self.B
        dev, T, H = md.device, y_seq.shape[2], md.d_hidden_Q
        L = _lib.lib()
        if md.training:
            raise ValueError("fused KNet step is inference only (model.eval())")
        S = getattr(self, "fs", None)
        if S is None or S["T"] != T:
            xm, xs, ym, ys = (t.reshape(-1).contiguous() for t in md._norm_tensors())
            um = None if md.u_mean is None else md.u_mean.reshape(-1).contiguous()
            us = None if md.u_std is None else md.u_std.reshape(-1).contiguous()
            z = lambda *sh: torch.zeros(sh, dtype=torch.float32, device=dev)   # noqa: E731
            G = max(1, min(self.groups, B))
            cuts = [B * g // G for g in range(G + 1)]
            S = {"T": T, "p": params_struct(md.sys.Params), "lim": limits_struct(md.sys.Params), "net": net_struct(md),
                 "norm": (xm, xs, ym, ys), "um": um, "us": us,
                 "y": z(B, md.n, T), "u": z(B, 2, T), "out": z(B, md.m, T), "post": z(B, md.m),
                 "hQ": z(B, H), "hSig": z(B, H), "hS": z(B, H), "prior": z(B, md.m), "dy": z(B, md.n),
                 "x2": z(B, 2 * H), "graph": None, "rows": list(zip(cuts[:-1], cuts[1:])),
                 "streams": [torch.cuda.Stream() for _ in range(G)] if G > 1 else []}
            nbytes = L.traj_knet_packed_bytes(C.byref(S["net"]))
            if nbytes == 0:
                raise NotImplementedError("fused KNet step: unsupported network shape")
            S["pk"] = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            S["ws"] = [torch.empty(L.traj_knet_fc2_workspace_bytes(C.byref(S["net"]), r1 - r0) // 4,
                                   dtype=torch.float32, device=dev) for r0, r1 in S["rows"]]
            _lib.check(L.traj_knet_pack_f32(C.byref(S["net"]), _p(S["pk"]), nbytes, _stream()), "traj_knet_pack_f32")
            self.fs = S

        def reset():
            S["y"].copy_(y_seq)
            S["u"].copy_(u_seq)
            for k in ("hQ", "hSig", "hS"):
                S[k].zero_()
            S["post"].copy_(m1x0.reshape(B, md.m))

        reset()
        if not use_graph:
            self._enqueue_all(T, T)
            return S["out"].clone()
        if S["graph"] is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self._enqueue_all(T, min(T, 2))   # warm up before capture
            torch.cuda.current_stream().wait_stream(s)
            reset()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._enqueue_all(T, T)
            S["graph"] = g
        S["graph"].replay()
        return S["out"].clone()

    @torch.no_grad()
    def run(self, y_seq, u_seq, m1x0, use_graph=True, fused=False):
        """y_seq [B,n,T] normalized, u_seq [B,2,T], m1x0 [B,m,1] -> posterior [B,m,T] (normalized).
        fused=True: the throughput path (eval mode; module state attributes are not updated)."""
        md = self.model
        if fused:
            return self._run_fused(y_seq, u_seq, m1x0, use_graph)
        T = y_seq.shape[2]
        out = torch.empty((self.B, md.m, T), device=md.device)
        if not use_graph:
            self._init_state(m1x0)
            for t in range(T):
                out[:, :, t] = md(y_seq[:, :, t:t + 1], u_seq[:, :, t:t + 1]).squeeze(2)
            return out
        # static-buffer form of the step for capture: the module's state tensors are updated in place
        self._init_state(m1x0)
        state = {"post": md.m1x_posterior.clone(), "hQ": md.h_Q.clone(), "hS": md.h_S.clone(),
                 "hSig": md.h_Sigma.clone()}

        def step():
            md.m1x_posterior, md.h_Q, md.h_S, md.h_Sigma = state["post"], state["hQ"], state["hS"], state["hSig"]
            r = md(self.y, self.u)
            state["post"].copy_(r)
            state["hQ"].copy_(md.h_Q)
            state["hS"].copy_(md.h_S)
            state["hSig"].copy_(md.h_Sigma)

        if self.graph is None:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):   # warm up the library GEMM paths before capture
                    step()
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                step()
            self.graph, self.state = g, state
        else:
            state = self.state
        # (re)initialize the captured state buffers
        self._init_state(m1x0)
        state["post"].copy_(md.m1x_posterior)
        state["hQ"].zero_()
        state["hS"].zero_()
        state["hSig"].zero_()
        for t in range(T):
            self.y.copy_(y_seq[:, :, t:t + 1])
            self.u.copy_(u_seq[:, :, t:t + 1])
            self.graph.replay()
            out[:, :, t] = state["post"].squeeze(2)
        return out


# --------------------------------------------------------------------------- EKF baseline (f2)
# R: generation_type1.py:24-32 measurement noise (phi not measured); Q: process noise of the Euler
# model, chosen for the synthetic data (the reference defines no EKF); P0: the initial-state spread.
EKF_R = (0.05 ** 2, 0.05 ** 2, 0.010 ** 2, 0.003 ** 2, 0.030 ** 2)
EKF_Q = (1e-6, 1e-6, 1e-5, 1e-4, 1e-4, 1e-2)
EKF_P0 = (0.1, 0.1, 0.1, 0.1, 0.01, 0.1)


def ekf_run(params: dict, Ts: float, y, u, x0, P0=EKF_P0, Q=EKF_Q, R=EKF_R):
    """Batched EKF over the clamped vehicle model (include/trajknet.h traj_ekf_run_f64), float64.
    y [B,5,T] real-unit measurements, u [B,2,T], x0 [B,6] -> estimates [B,6,T]."""
    dev = require_gpu(y.device if torch.is_tensor(y) and y.is_cuda else None)
    f64 = lambda a: torch.as_tensor(a, dtype=torch.float64, device=dev).contiguous()   # noqa: E731
    yy, uu, xx = f64(y), f64(u), f64(x0).reshape(-1, 6)
    B, T = yy.shape[0], yy.shape[2]
    out = torch.empty((B, 6, T), dtype=torch.float64, device=dev)
    p0, q, r = f64(P0), f64(Q), f64(R)     # kept alive until the launch is enqueued
    _lib.check(_lib.lib().traj_ekf_run_f64(C.byref(params_struct(params)), C.byref(limits_struct(params)), float(Ts),
                                           B, T, _p(yy), _p(uu), _p(xx), _p(p0), _p(q), _p(r), _p(out),
                                           _stream()), "traj_ekf_run_f64")
    return out


# torch.ops.trajknet.* (prior, gru_gates, update, pack, step): the same HIP ops registered with torch.library
from . import knet_ops  # noqa: E402,F401
