"""KalmanNet training step on MI355X: drop-in for KalmanNet/pipeline.py's loss
functions and ``train_epoch`` (:14-181).

The forward is the module path of ``knet.KalmanNetNN`` (HIP prior / GRU-gate / update ops under
autograd, GEMMs on hipBLASLt); the backward differentiates the reference's own expressions on the
device (``knet.torch_prior``, ``knet.torch_gru_gates``); clipping and the optimizer are torch's.
Truncated BPTT as the reference runs it: a loss and a backward every ``K_TBPTT`` steps, then either an
optimizer step per chunk (``'standard'``) or one per trajectory (``'accumulation'``), and the hidden
states / posterior detached at every chunk end.
"""
from __future__ import annotations

import random

import torch
from torch.nn.utils import clip_grad_norm_

PHI_IDX = 2      # pipeline.py:11
EPS_DB = 1e-12   # pipeline.py:12


def _angular_mse_from_real(phi_pred_real, phi_tgt_real):
    """pipeline.py:16-20: MSE of the wrapped angle difference."""
    diff = torch.atan2(torch.sin(phi_pred_real - phi_tgt_real), torch.cos(phi_pred_real - phi_tgt_real))
    return (diff ** 2).mean()


def loss_x_with_angular(x_out_norm, x_tgt_norm, x_mean, x_std, m, phi_idx=PHI_IDX):
    """pipeline.py:22-41: (m-1)/m * MSE of the non-phi channels (normalized) + 1/m * angular MSE of phi
    (denormalized)."""
    diff2 = (x_out_norm - x_tgt_norm) ** 2
    idx_no_phi = [i for i in range(m) if i != phi_idx]
    mse_no_phi = diff2[:, idx_no_phi, :].mean()
    x_out_real = (x_out_norm * x_std) + x_mean
    x_tgt_real = (x_tgt_norm * x_std) + x_mean
    mse_phi_ang = _angular_mse_from_real(x_out_real[:, phi_idx, :], x_tgt_real[:, phi_idx, :])
    return (float(m - 1) / m) * mse_no_phi + (1.0 / m) * mse_phi_ang


def compute_composite_loss(x_out_norm, x_tgt_norm, y_tgt_norm, x_mean, x_std, m, n, alpha, phi_idx=PHI_IDX):
    """pipeline.py:44-60: alpha * state loss + (1 - alpha) * MSE of the observed channels against y."""
    loss_x = loss_x_with_angular(x_out_norm, x_tgt_norm, x_mean, x_std, m, phi_idx)
    idx_y = [i for i in range(m) if i != phi_idx]
    loss_y = torch.nn.functional.mse_loss(x_out_norm[:, idx_y, :], y_tgt_norm, reduction="mean")
    return alpha * loss_x + (1.0 - alpha) * loss_y


def tbptt_sequence(model, optimizer, y_norm, u, x_norm, m1x0, params, x_mean, x_std):
    """The body of train_epoch (pipeline.py:94-181) for one batch already on the device: normalized
    observations y_norm [B,n,T], controls u [B,2,T], normalized targets x_norm [B,m,T], initial
    posterior m1x0 [B,m,1].  Returns (mean chunk loss, its dB value, per-chunk losses)."""
    strategy, K, T = params["strategy"], params["K_TBPTT"], params["T"]
    m, n = params["m"], params["n"]
    use_composite, alpha = params["CompositionLoss"], params["alpha"]
    B = y_norm.shape[0]
    model.batch_size = B
    model.init_hidden_KNet()
    model.InitSequence(m1x0, T)
    optimizer.zero_grad()
    num_chunks = (T + K - 1) // K
    outs, xt, yt, losses = [], [], [], []
    for t in range(T):
        x_out = model(y_norm[:, :, t].unsqueeze(2), u[:, :, t].unsqueeze(2))
        outs.append(x_out.squeeze(2))
        xt.append(x_norm[:, :, t])
        if use_composite:
            yt.append(y_norm[:, :, t])
        if ((t + 1) % K == 0) or (t + 1 == T):
            xo, xg = torch.stack(outs, dim=2), torch.stack(xt, dim=2)
            if use_composite:
                loss = compute_composite_loss(xo, xg, torch.stack(yt, dim=2), x_mean, x_std, m, n, alpha, PHI_IDX)
            else:
                loss = loss_x_with_angular(xo, xg, x_mean, x_std, m, PHI_IDX)
            if strategy == "accumulation":
                (loss / num_chunks).backward()
            else:
                loss.backward()
                clip_grad_norm_(model.parameters(), max_norm=5.0)
                optimizer.step()
                optimizer.zero_grad()
            losses.append(float(loss.item()))
            outs, xt, yt = [], [], []
            model.h_Q = model.h_Q.detach()
            model.h_Sigma = model.h_Sigma.detach()
            model.h_S = model.h_S.detach()
            model.m1x_posterior = model.m1x_posterior.detach()
    if strategy == "accumulation":
        clip_grad_norm_(model.parameters(), max_norm=5.0)
        optimizer.step()
        optimizer.zero_grad()
    avg = sum(losses) / max(1, len(losses))
    loss_db = 10 * torch.log10(torch.tensor(avg).clamp_min(EPS_DB))
    return avg, loss_db, losses


def train_epoch(model, optimizer, y_train, u_train, x_train, norm_stats, params):
    """pipeline.py:63-181: one training step on a random batch of N_batch of the N_E trajectories
    (y/u/x [N_E, c, T] real units), initial posterior = normalized x(0) + N(0, 0.2^2) noise.
    Returns (average chunk loss, loss in dB)."""
    device = params["device"]
    x_mean, x_std = norm_stats["x_mean"].to(device), norm_stats["x_std"].to(device)
    model.train()
    indices = random.sample(range(params["N_E"]), k=params["N_batch"])
    y_b, u_b, x_b = (t[indices].to(device) for t in (y_train, u_train, x_train))
    y_norm = (y_b - norm_stats["y_mean"].to(device)) / norm_stats["y_std"].to(device)
    x_norm = (x_b - x_mean) / x_std
    x0 = x_norm[:, :, 0]
    m1x0 = (x0 + torch.randn_like(x0) * 0.2).unsqueeze(2)
    avg, loss_db, _ = tbptt_sequence(model, optimizer, y_norm, u_b, x_norm, m1x0, params, x_mean, x_std)
    return avg, loss_db
