"""KalmanNet vs the EKF baseline on the same noisy sequences (BASELINE.json configs[4]: 1024 sequences x
200 steps, Ts = 0.01, "MSE vs reference EKF").

The evaluation is KalmanNet/test_vehicle.py's, on data this build generates:

  * sequences: the closed-loop MPC trajectories of the dataset emitter (batch.run_closed_loop, spline
    references, plant step Ts) with the reference's measurement noise (dataset.measurement_noise =
    generation_type1.py:312-320), cut to the first T rows as data_loader.py:14-53 does: observations
    y = noisy [X, Y, vx, vy, omega], inputs u = [d, delta], targets x = clean states, float32 [B, C, T];
  * normalization from a separate "train" draw (ids offset by TRAIN_ID_OFFSET): mean / std over
    (sequence, time) + 1e-8, and the clamp limits of vehicle_model.py as the train states' min / max
    (test_vehicle.py:76-92);
  * KalmanNet initialized with the hybrid initial posterior of test_vehicle.py:123-133 (measured
    channels of y_0 in normalized space, phi = 0);
  * the loss of test_vehicle.py:15-40 (= pipeline.py:16-41, knet_train.loss_x_with_angular): MSE of
    the non-phi channels in normalized space plus the wrapped-angle MSE of phi in real units, and its
    dB value (test_vehicle.py:149-158);
  * the EKF (knet.ekf_run, traj_ekf_run_f64) on the same measurements and inputs, started from the same
    hybrid posterior in real units, scored with the same loss after normalization.

The reference ships no trained weights and no EKF; the KalmanNet figures are for whatever weights the
model holds (the bench: the seeded init of the reference architecture, so its MSE is that of an
untrained filter).
"""
from __future__ import annotations

import numpy as np
import torch

from . import batch as TB
from .dataset import measurement_noise
from .knet_train import EPS_DB, PHI_IDX, loss_x_with_angular
from .workload import make_workload

TRAIN_ID_OFFSET = 1 << 20   # ids of the normalization ("train") draw: disjoint from the test ids
OBS_IDX = (0, 1, 3, 4, 5)   # vehicle_model.py:149-150 (h), data_loader.py noisy columns


def make_sequences(B, T, Ts=0.01, N=20, seed=0, id_offset=0, device=None):
    """B closed-loop trajectories of T rows at plant step Ts -> dict of float32 tensors y [B,5,T]
    (noisy, real units), u [B,2,T], x [B,6,T] (clean), on the GPU."""
    w = make_workload(B, N, Ts, kind="spline", seed=seed, id_offset=id_offset)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=device)
    res = TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, TB.config_struct(N=N, Ts=Ts))
    X = res["X"][:, :T]                                    # rows 0 .. T-1 (data_loader.py:41-53)
    U = res["U"][:, :T]
    noise = np.stack([measurement_noise(int(i), T + 1)[:T] for i in w["ids"]])
    Xn = X + torch.as_tensor(noise, device=X.device)
    f32 = lambda a: a.permute(0, 2, 1).contiguous().to(torch.float32)   # noqa: E731  [B,T,C] -> [B,C,T]
    return {"y": f32(Xn[:, :, list(OBS_IDX)]), "u": f32(U), "x": f32(X),
            "status": res["status"], "ids": w["ids"]}


def normalization(train):
    """test_vehicle.py:76-92: (x_mean, x_std, y_mean, y_std) as [1,C,1] and the 12 clamp limits."""
    x, y = train["x"], train["y"]
    m, n = x.shape[1], y.shape[1]
    xm = x.mean(dim=(0, 2)).reshape(1, m, 1)
    xs = x.std(dim=(0, 2)).reshape(1, m, 1) + 1e-8
    ym = y.mean(dim=(0, 2)).reshape(1, n, 1)
    ys = y.std(dim=(0, 2)).reshape(1, n, 1) + 1e-8
    lim = {}
    for i, k in enumerate(("x", "y", "phi", "vx", "vy", "omega")):
        lim[f"{k}_min"] = float(x[:, i, :].min())
        lim[f"{k}_max"] = float(x[:, i, :].max())
    return xm, xs, ym, ys, lim


def hybrid_init(y_norm, m=6):
    """test_vehicle.py:123-133: the measured channels of y_0 (normalized), phi = 0 -> [B,m,1]."""
    B = y_norm.shape[0]
    m1x0 = torch.zeros(B, m, 1, device=y_norm.device, dtype=y_norm.dtype)
    for j, i in enumerate(OBS_IDX):
        m1x0[:, i, 0] = y_norm[:, j, 0]
    return m1x0


def mse_and_db(x_out_norm, x_tgt_norm, xm, xs, m=6):
    """test_vehicle.py:143-158: the angular state loss and 10 log10(max(loss, 1e-12))."""
    loss = float(loss_x_with_angular(x_out_norm.float(), x_tgt_norm.float(), xm, xs, m, PHI_IDX))
    return loss, float(10.0 * np.log10(max(loss, EPS_DB)))


def ekf_vs_truth(params, Ts, test, xm, xs, ym, ys):
    """EKF (knet.ekf_run) on the test measurements from the hybrid initial posterior (real units);
    returns (normalized estimates [B,6,T], loss, dB)."""
    from .knet import ekf_run
    y_norm = (test["y"] - ym) / ys
    x0 = (hybrid_init(y_norm) * xs + xm).squeeze(2)
    est = ekf_run(params, Ts, test["y"].double(), test["u"].double(), x0.double())
    est_norm = (est.float() - xm) / xs
    loss, db = mse_and_db(est_norm, (test["x"] - xm) / xs, xm, xs)
    return est_norm, loss, db
