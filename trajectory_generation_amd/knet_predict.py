"""Sliding-window open-loop prediction evaluation of a KalmanNet filter (KalmanNet/test_prediction.py) on
the device.

The reference scores a trained filter trajectory by trajectory: run the filter over the whole sequence
at batch size 1 (run_full_filter, :45-65), then from every EVAL_STEP-th estimate roll the vehicle model
H steps open loop with the logged inputs (rollout_open_loop, :67-87) and measure the XY error against the
ground truth (compute_metrics / get_error_profile, :89-112; window loop :172-235).  Here the same
evaluation runs for all trajectories at once:

  * the filter: KNetSequenceRunner's fused step over the B trajectories (one graph of T steps);
  * the rollouts: every (trajectory, window) pair in one launch of traj_knet_rollout_eval_f32 (one
    thread per window; H clamped Euler steps of the same float32 physics as the filter's prior), which
    also produces each window's ADE / FDE and error profile;
  * the initial states: test_prediction.py:172,184-193 ("noisy_gt": the normalized first state plus
    INIT_NOISE_STD x N(0, 1), drawn per trajectory in order from a CPU generator seeded with INIT_SEED --
    the reference's draws when it runs on the CPU).

Names and argument meanings follow the reference's functions; the plotting of main() (:238-362) is out of
scope.  Figures are float32 like the reference; ADE is accumulated in float64 inside the kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _lib
from .batch import params_struct, require_gpu
from .knet import KalmanNetNN, KNetSequenceRunner, limits_struct

H_PRED = 200          # test_prediction.py:31
EVAL_STEP = 100       # :32
T_START_EVAL = 50     # :33
INIT_MODE = "noisy_gt"   # :40
INIT_NOISE_STD = 0.2     # :41
INIT_SEED = 0            # :42


def _p(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def init_states(x_gt, x_mean, x_std, mode=INIT_MODE, noise_std=INIT_NOISE_STD, seed=INIT_SEED):
    """test_prediction.py:172,184-193 for B trajectories: x_gt [B,6,T] real, x_mean / x_std [1,6,1] ->
    x0n [B,6,1] normalized.  The noise of trajectory i is the i-th [1,6] draw of a CPU generator seeded
    once with `seed`, as the reference's loop draws it."""
    xm = x_mean.reshape(1, 6).to(x_gt.device, torch.float32)
    xs = x_std.reshape(1, 6).to(x_gt.device, torch.float32)
    x0 = (x_gt[:, :, 0].float() - xm) / xs
    if mode == "gt":
        return x0.unsqueeze(2)
    if mode != "noisy_gt":
        raise ValueError("Invalid INIT_MODE")
    g = torch.Generator().manual_seed(seed)
    noise = torch.cat([torch.randn((1, 6), generator=g) for _ in range(x_gt.shape[0])], 0)
    return (x0 + noise.to(x0.device) * noise_std).unsqueeze(2)


@torch.no_grad()
def run_full_filter(model: KalmanNetNN, y_norm, u, x0_norm, runner: KNetSequenceRunner | None = None):
    """test_prediction.py:45-65 for B trajectories at once: y_norm [B,5,T], u [B,2,T], x0_norm [B,6,1] ->
    the normalized estimates [B,6,T] (the fused sequence runner; the model must be in eval mode)."""
    model.eval()
    B = y_norm.shape[0]
    if runner is None or runner.B != B:
        runner = KNetSequenceRunner(model, B)
    return runner.run(y_norm.float().contiguous(), u.float().contiguous(), x0_norm.float(), fused=True)


def _launch(sys_model, B, T, H, t0, step, nwin, x_est, strides, norm, u, x_gt, ade, fde, prof, pred):
    L = _lib.lib()
    xm, xs = norm
    _lib.check(L.traj_knet_rollout_eval_f32(
        C.byref(params_struct(sys_model.Params)), C.byref(limits_struct(sys_model.Params)), float(sys_model.Ts),
        B, T, H, t0, step, nwin, _p(x_est), *strides, _p(xm), _p(xs), _p(u), _p(x_gt), _p(ade), _p(fde),
        _p(prof), _p(pred), _stream()), "traj_knet_rollout_eval_f32")


@torch.no_grad()
def rollout_open_loop(sys_model, x0_real, u, t_start_state, H):
    """test_prediction.py:67-87: x0_real [B,6,1] (real units), u [B,2,T] -> the H' = min(H, T - t_start)
    predicted states [B,6,H'] (x0_real itself when H' = 0, the reference's fallback)."""
    require_gpu()
    dev = x0_real.device
    B, T = x0_real.shape[0], u.shape[2]
    Hs = max(0, min(H, T - t_start_state))
    if Hs == 0:
        return x0_real
    x0 = x0_real.reshape(B, 6).float().contiguous()
    uu = u.float().contiguous()
    pred = torch.empty((B, 6, Hs), dtype=torch.float32, device=dev)
    _launch(sys_model, B, T, Hs, t_start_state, 1, 1, x0, (6, 1, 0), (None, None), uu, None, None, None, None, pred)
    return pred


def compute_metrics(pred_real, gt_real):
    """test_prediction.py:89-103: ADE and FDE on XY of one window ([1,m,H] each) as Python floats."""
    err = torch.sqrt(torch.sum((pred_real[:, :2, :] - gt_real[:, :2, :]) ** 2, dim=1))
    return err.mean().item(), err[0, -1].item()


def get_error_profile(pred_real, gt_real):
    """test_prediction.py:105-112: the XY error per step of one window as a numpy array [H]."""
    err = torch.sqrt(torch.sum((pred_real[:, :2, :] - gt_real[:, :2, :]) ** 2, dim=1))
    return err.squeeze(0).cpu().numpy()


@torch.no_grad()
def window_scores(sys_model, x_est_norm, x_mean, x_std, u, x_gt, H=H_PRED, eval_step=EVAL_STEP,
                  t_start=T_START_EVAL, profile=True):
    """The window loop of test_prediction.py:199-221 for B trajectories in one launch: windows t in
    range(t_start, T - H, eval_step) of every trajectory, each rolled out from x_est_norm[:, :, t] *
    x_std + x_mean.  Returns ade [B,W], fde [B,W] and (profile=True) the error profiles [B,W,H]."""
    require_gpu()
    dev = x_est_norm.device
    B, T = x_est_norm.shape[0], x_est_norm.shape[2]
    nwin = _lib.lib().traj_knet_rollout_windows(T, H, t_start, eval_step)
    if nwin < 0:
        raise ValueError("window_scores: need H >= 1, t_start >= 0, eval_step >= 1")
    xe = x_est_norm.float().contiguous()
    xm = x_mean.reshape(6).to(dev, torch.float32).contiguous()
    xs = x_std.reshape(6).to(dev, torch.float32).contiguous()
    uu, xg = u.float().contiguous(), x_gt.float().contiguous()
    if uu.shape != (B, 2, T) or xg.shape != (B, 6, T) or xe.shape != (B, 6, T):
        raise ValueError("window_scores: x_est_norm [B,6,T], u [B,2,T] and x_gt [B,6,T] must match")
    ade = torch.empty((B, nwin), dtype=torch.float32, device=dev)
    fde = torch.empty_like(ade)
    prof = torch.empty((B, nwin, H), dtype=torch.float32, device=dev) if profile else None
    _launch(sys_model, B, T, H, t_start, eval_step, nwin, xe, (6 * T, T, 1), (xm, xs), uu, xg, ade, fde, prof, None)
    return ade, fde, prof


@torch.no_grad()
def sliding_window_eval(model: KalmanNetNN, sys_model, y, u, x_gt, x_mean, x_std, y_mean, y_std, H=H_PRED,
                        eval_step=EVAL_STEP, t_start=T_START_EVAL, init_mode=INIT_MODE,
                        init_noise_std=INIT_NOISE_STD, init_seed=INIT_SEED, runner=None):
    """test_prediction.py:166-235 for the whole test set: y [B,5,T] (real), u [B,2,T], x_gt [B,6,T] (real),
    normalization statistics [1,C,1].  Returns the per-window arrays and main()'s printed summary
    (mean / std of ADE and FDE over all windows, the mean / std error profile of :271-275)."""
    dev = model.device
    y, u, x_gt = (t.to(dev, torch.float32) for t in (y, u, x_gt))
    ym = y_mean.reshape(1, 5, 1).to(dev, torch.float32)
    ys = y_std.reshape(1, 5, 1).to(dev, torch.float32)
    y_norm = (y - ym) / ys                                                   # :183
    x0n = init_states(x_gt, x_mean, x_std, init_mode, init_noise_std, init_seed)
    x_est = run_full_filter(model, y_norm, u, x0n, runner)
    ade, fde, prof = window_scores(sys_model, x_est, x_mean, x_std, u, x_gt, H, eval_step, t_start)
    a = ade.double().cpu().numpy().reshape(-1)
    f = fde.double().cpu().numpy().reshape(-1)
    P = prof.double().cpu().numpy().reshape(-1, H)
    return {"x0n": x0n, "x_est": x_est, "ade": ade, "fde": fde, "profile": prof,
            "n_windows": int(a.size), "horizon": H, "horizon_s": H * float(sys_model.Ts),
            "ade_mean": float(np.mean(a)) if a.size else float("nan"), "ade_std": float(np.std(a)) if a.size else 0.0,
            "fde_mean": float(np.mean(f)) if f.size else float("nan"), "fde_std": float(np.std(f)) if f.size else 0.0,
            "err_time_mean": P.mean(0) if a.size else np.zeros(H), "err_time_std": P.std(0) if a.size else np.zeros(H)}
