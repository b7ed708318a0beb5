"""CPU restatement of the KalmanNet inference step -- TEST INFRASTRUCTURE ONLY (tests/, bench.py's
cpu_baseline leg).  Never imported by the product package.

Follows, in float32 like the reference (torch CPU tensors, functional form):
  KalmanNet/vehicle_model.py:19-42   pt_tire_forces (KNet variant: vx_eff = max(|vx|, vx_zero), only
                                     alpha_f clamped, Frx on vx_eff)
  KalmanNet/vehicle_model.py:45-79   pt_f_cont (phi, vx, vy, omega clamped to the data limits first)
  KalmanNet/vehicle_model.py:109-153 f (Euler step, all six states clamped), h (rows 0,1,3,4,5)
  KalmanNet/kalman_net.py:145-216    step_prior, KGain_step, KNet_step (eval mode: dropout = identity)
  torch.nn.GRU (seq_len 1)           r = s(W_ir x + b_ir + W_hr h + b_hr), z likewise,
                                     n = tanh(W_in x + b_in + r (W_hn h + b_hn)), h' = (1 - z) n + z h
Pinned to the reference by tests/golden/knet.npz (tests/golden/gen_knet_golden.py).
"""
from __future__ import annotations

import math

import torch

PARAMS = {"Cm1": 0.287, "Cm2": 0.0545, "Cr0": 0.0518, "Cr2": 0.00035, "Br": 3.3852, "Cr": 1.2691, "Dr": 0.1737,
          "Bf": 2.579, "Cf": 1.2, "Df": 0.192, "m": 0.041, "Iz": 27.8e-6, "lf": 0.029, "lr": 0.033, "g": 9.81,
          "maxAlpha": 0.6, "vx_zero": 0.3}


def f_cont(x, u, p):
    """x [B,6], u [B,2] -> x_dot [B,6] (vehicle_model.py:45-79)."""
    phi = torch.clamp(x[:, 2], p["phi_min"], p["phi_max"])
    vx = torch.clamp(x[:, 3], p["vx_min"], p["vx_max"])
    vy = torch.clamp(x[:, 4], p["vy_min"], p["vy_max"])
    om = torch.clamp(x[:, 5], p["omega_min"], p["omega_max"])
    d, de = u[:, 0], u[:, 1]
    vx_eff = torch.maximum(vx.abs(), torch.full_like(vx, p["vx_zero"]))
    af = -torch.atan2(om * p["lf"] + vy, vx_eff) + de
    ar = torch.atan2(om * p["lr"] - vy, vx_eff)
    af = torch.clamp(af, -p["maxAlpha"], p["maxAlpha"])
    Fyf = p["Df"] * torch.sin(p["Cf"] * torch.atan(p["Bf"] * af))
    Fyr = p["Dr"] * torch.sin(p["Cr"] * torch.atan(p["Br"] * ar))
    Frx = (p["Cm1"] - p["Cm2"] * vx_eff) * d - p["Cr0"] - p["Cr2"] * (vx_eff * vx_eff)
    return torch.stack([vx * torch.cos(phi) - vy * torch.sin(phi), vx * torch.sin(phi) + vy * torch.cos(phi), om,
                        (Frx - Fyf * torch.sin(de) + p["m"] * vy * om) / p["m"],
                        (Fyr + Fyf * torch.cos(de) - p["m"] * vx * om) / p["m"],
                        (Fyf * p["lf"] * torch.cos(de) - Fyr * p["lr"]) / p["Iz"]], 1)


def f_step(x, u, p, Ts):
    """vehicle_model.py:109-134 on [B,6] / [B,2]."""
    xn = x + Ts * f_cont(x, u, p)
    keys = (("x_min", "x_max"), ("y_min", "y_max"), ("phi_min", "phi_max"), ("vx_min", "vx_max"),
            ("vy_min", "vy_max"), ("omega_min", "omega_max"))
    return torch.stack([torch.clamp(xn[:, i], p[lo], p[hi]) for i, (lo, hi) in enumerate(keys)], 1)


def h(x):
    return x[:, [0, 1, 3, 4, 5]]


def _lin(x, W, b, relu=True):
    y = x @ W.t() + b
    return torch.relu(y) if relu else y


def _gru(x, hprev, w, name):
    gi = x @ w[f"{name}.weight_ih_l0"].t() + w[f"{name}.bias_ih_l0"]
    gh = hprev @ w[f"{name}.weight_hh_l0"].t() + w[f"{name}.bias_hh_l0"]
    H = hprev.shape[1]
    r = torch.sigmoid(gi[:, :H] + gh[:, :H])
    z = torch.sigmoid(gi[:, H:2 * H] + gh[:, H:2 * H])
    n = torch.tanh(gi[:, 2 * H:] + r * gh[:, 2 * H:])
    return (1 - z) * n + z * hprev


def run_sequences(weights, p, Ts, y_norm, u, m1x0, x_mean, x_std, y_mean, y_std, hidden=128):
    """weights: state_dict-like dict of float32 tensors; y_norm [B,5,T], u [B,2,T], m1x0 [B,6,1];
    means/stds [1,6,1] / [1,5,1].  Returns the normalized posteriors [B,6,T]."""
    w = {k: torch.as_tensor(v, dtype=torch.float32) for k, v in weights.items()}
    f32 = lambda a: torch.as_tensor(a, dtype=torch.float32)   # noqa: E731
    y_norm, u, m1x0 = f32(y_norm), f32(u), f32(m1x0)
    xm, xs, ym, ys = (f32(a).reshape(1, -1) for a in (x_mean, x_std, y_mean, y_std))
    B, T = y_norm.shape[0], y_norm.shape[2]
    post = m1x0.reshape(B, 6)
    hQ = torch.zeros(B, hidden)
    hSig = torch.zeros(B, hidden)
    hS = torch.zeros(B, hidden)
    gamma = torch.sigmoid(w["innov_logit"])
    out = torch.empty(B, 6, T)
    for t in range(T):
        x_real = post * xs + xm
        x_prior_real = f_step(x_real, u[:, :, t], p, Ts)
        prior = (x_prior_real - xm) / xs
        m1y = (h(x_prior_real) - ym) / ys
        dy = y_norm[:, :, t] - m1y
        o5 = _lin(prior, w["FC5.0.weight"], w["FC5.0.bias"])
        hQ = _gru(o5, hQ, w, "GRU_Q")
        oSig = _gru(hQ, hSig, w, "GRU_Sigma")
        o1 = _lin(oSig, w["FC1.0.weight"], w["FC1.0.bias"])
        o7 = _lin(dy, w["FC7.0.weight"], w["FC7.0.bias"])
        hS = _gru(torch.cat((o1, o7), 1), hS, w, "GRU_S")
        o2 = _lin(_lin(torch.cat((oSig, hS), 1), w["FC2.0.weight"], w["FC2.0.bias"]), w["FC2.2.weight"],
                  w["FC2.2.bias"], relu=False)
        o3 = _lin(torch.cat((hS, o2), 1), w["FC3.0.weight"], w["FC3.0.bias"])
        hSig = _lin(torch.cat((oSig, o3), 1), w["FC4.0.weight"], w["FC4.0.bias"])
        KG = o2.reshape(B, 6, 5)
        post = prior + gamma * torch.bmm(KG, dy.unsqueeze(2)).squeeze(2)
        out[:, :, t] = post
    return out


def angular_mse_db(x_est_real, x_true_real, phi_idx=2):
    """MSE [dB] with the heading error wrapped (test_vehicle.py:15-40, :149-158 style)."""
    d = x_est_real - x_true_real
    d[:, phi_idx] = torch.atan2(torch.sin(d[:, phi_idx]), torch.cos(d[:, phi_idx]))
    return 10.0 * math.log10(float((d ** 2).mean()) + 1e-12)


# ------------------------------------------------------------------ sliding-window prediction scoring
# KalmanNet/test_prediction.py: rollout_open_loop :67-87, compute_metrics :89-103, get_error_profile
# :105-112 and the window loop of main() :176-221, in float32 on CPU tensors.

def rollout_open_loop(x0_real, u, t_start, H, p, Ts):
    """x0_real [B,6], u [B,2,T] -> predicted states [B,6,H'] (H' = min(H, T - t_start); :67-87)."""
    x, preds = x0_real, []
    for k in range(H):
        tu = t_start + k
        if tu >= u.shape[2]:
            break
        x = f_step(x, u[:, :, tu], p, Ts)
        preds.append(x)
    return torch.stack(preds, 2) if preds else x0_real.unsqueeze(2)


def error_profile(pred_real, gt_real):
    """[B,6,H] x2 -> XY Euclidean error per step [B,H] (:95-98, :110-111)."""
    diff = pred_real[:, :2, :] - gt_real[:, :2, :]
    return torch.sqrt(torch.sum(diff ** 2, dim=1))


def sliding_window_scores(x_est_norm, x_mean, x_std, u, x_gt, p, Ts, H, step, t0):
    """main()'s window loop (:199-221) for B sequences at once: windows t in range(t0, T - H, step), the
    rollout from the filter estimate x_est_norm[:, :, t] * x_std + x_mean (:202-203) scored against
    x_gt[:, :, t+1 : t+1+H].  Returns ade [B, W], fde [B, W], profile [B, W, H] (float32)."""
    f32 = lambda a: torch.as_tensor(a, dtype=torch.float32)   # noqa: E731
    x_est_norm, u, x_gt = f32(x_est_norm), f32(u), f32(x_gt)
    xm, xs = f32(x_mean).reshape(1, 6), f32(x_std).reshape(1, 6)
    T = x_est_norm.shape[2]
    ades, fdes, profs = [], [], []
    for t in range(t0, T - H, step):
        x_start = x_est_norm[:, :, t] * xs + xm
        pred = rollout_open_loop(x_start, u, t, H, p, Ts)
        e = error_profile(pred, x_gt[:, :, t + 1:t + 1 + H])
        ades.append(e.mean(1))
        fdes.append(e[:, -1])
        profs.append(e)
    if not ades:
        B = x_est_norm.shape[0]
        return torch.zeros(B, 0), torch.zeros(B, 0), torch.zeros(B, 0, H)
    return torch.stack(ades, 1), torch.stack(fdes, 1), torch.stack(profs, 1)


# ------------------------------------------------------------------ EKF baseline (no reference
# counterpart: SURVEY.md 8(f) f2); the same algorithm as include/trajknet.h traj_ekf_run_f64, float64.
def _veh_f64(x, d, de, p, Ts):
    lo = [p["x_min"], p["y_min"], p["phi_min"], p["vx_min"], p["vy_min"], p["omega_min"]]
    hi = [p["x_max"], p["y_max"], p["phi_max"], p["vx_max"], p["vy_max"], p["omega_max"]]
    cl = lambda v, i: min(max(v, lo[i]), hi[i])   # noqa: E731
    phi, vx, vy, om = cl(x[2], 2), cl(x[3], 3), cl(x[4], 4), cl(x[5], 5)
    vx_eff = max(abs(vx), p["vx_zero"])
    af = -math.atan2(om * p["lf"] + vy, vx_eff) + de
    ar = math.atan2(om * p["lr"] - vy, vx_eff)
    af = min(max(af, -p["maxAlpha"]), p["maxAlpha"])
    Fyf = p["Df"] * math.sin(p["Cf"] * math.atan(p["Bf"] * af))
    Fyr = p["Dr"] * math.sin(p["Cr"] * math.atan(p["Br"] * ar))
    Frx = (p["Cm1"] - p["Cm2"] * vx_eff) * d - p["Cr0"] - p["Cr2"] * (vx_eff * vx_eff)
    sp, cp, sd, cd = math.sin(phi), math.cos(phi), math.sin(de), math.cos(de)
    xd = [vx * cp - vy * sp, vx * sp + vy * cp, om, (Frx - Fyf * sd + p["m"] * vy * om) / p["m"],
          (Fyr + Fyf * cd - p["m"] * vx * om) / p["m"], (Fyf * p["lf"] * cd - Fyr * p["lr"]) / p["Iz"]]
    return [cl(x[i] + Ts * xd[i], i) for i in range(6)]


def ekf_run(p, Ts, y, u, x0, P0, Q, R):
    """y [B,5,T], u [B,2,T], x0 [B,6] (numpy) -> [B,6,T]."""
    import numpy as np
    y, u, x0 = np.asarray(y, float), np.asarray(u, float), np.asarray(x0, float)
    B, T = y.shape[0], y.shape[2]
    H = np.zeros((5, 6))
    for a, r in enumerate((0, 1, 3, 4, 5)):
        H[a, r] = 1.0
    out = np.zeros((B, 6, T))
    for b in range(B):
        x = x0[b].copy()
        P = np.diag(P0)
        for t in range(T):
            d, de = u[b, 0, t], u[b, 1, t]
            xm = np.array(_veh_f64(x, d, de, p, Ts))
            F = np.zeros((6, 6))
            for j in range(6):
                h = 1e-6 * max(1.0, abs(x[j]))
                xp, xq = x.copy(), x.copy()
                xp[j] += h
                xq[j] -= h
                F[:, j] = (np.array(_veh_f64(xp, d, de, p, Ts)) - np.array(_veh_f64(xq, d, de, p, Ts))) / (2 * h)
            Pm = F @ P @ F.T + np.diag(Q)
            S = H @ Pm @ H.T + np.diag(R)
            K = np.linalg.solve(S, H @ Pm).T
            x = xm + K @ (y[b, :, t] - H @ xm)
            A = np.eye(6) - K @ H
            P = A @ Pm @ A.T + K @ np.diag(R) @ K.T
            out[b, :, t] = x
    return out
