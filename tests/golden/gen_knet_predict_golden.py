"""Generate tests/golden/knet_predict.npz -- the sliding-window prediction scores of the REFERENCE's own
KalmanNet/test_prediction.py functions.

Run in the build container only (reads /root/reference):  python tests/golden/gen_knet_predict_golden.py

Imported read-only from /root/reference/KalmanNet: test_prediction (run_full_filter :45-65,
rollout_open_loop :67-87, compute_metrics :89-103, get_error_profile :105-112; imported from a scratch
working directory because the module creates its results directory at import, with matplotlib's Agg
backend), kalman_net.KalmanNetNN and vehicle_model.VehicleModel.  The window loop is main()'s
(:172-221: torch.manual_seed(INIT_SEED) once, then per trajectory the noisy_gt initial state, the full
filter, and windows t in range(T_START_EVAL, T - H, EVAL_STEP)); main() itself needs the dataset CSVs and
a trained weight file, so the loop is driven here with the same calls on synthetic data.  The network is
test_prediction's architecture (in_mult 10, :149) with the deterministic weights of tests/_knet_weights.py.
Sizes are scaled down (B = 3 trajectories of T = 90 steps, H = 20, EVAL_STEP = 15, T_START_EVAL = 10)
so the CPU reference finishes in seconds.
"""
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests._knet_weights import LIMITS, knet_weights  # noqa: E402

REF = "/root/reference/KalmanNet"
B, T, H, EVAL_STEP, T_START, Ts = 3, 90, 20, 15, 10, 0.01
IN_MULT, SEED_W, INIT_SEED, INIT_NOISE_STD = 10, 3, 0, 0.2


def main():
    os.environ.setdefault("MPLBACKEND", "Agg")
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as scratch:
        os.chdir(scratch)
        try:
            import test_prediction as TP
        finally:
            os.chdir(cwd)
    import kalman_net as KN
    import vehicle_model as VM
    torch.set_num_threads(4)
    rng = np.random.default_rng(11)
    dummy = torch.eye(6)
    sysm = VM.VehicleModel(Ts, T, T, torch.zeros(6, 1), dummy, dummy, torch.eye(5))
    params = dict(VM.Params)
    params.update(LIMITS)
    sysm.Params = params

    # synthetic trajectories simulated with the reference model (controls piecewise smooth)
    x = np.stack([rng.uniform(0, 2, B), rng.uniform(-0.5, 0.5, B), rng.uniform(-0.3, 0.3, B),
                  rng.uniform(0.8, 1.6, B), rng.uniform(-0.05, 0.05, B), rng.uniform(-0.5, 0.5, B)], 1)
    X, U = [x], []
    for t in range(T):
        u = np.stack([0.25 + 0.15 * np.sin(0.05 * t + np.arange(B)), 0.2 * np.sin(0.03 * t + 2.0 * np.arange(B))], 1)
        xn = sysm.f(torch.tensor(X[-1], dtype=torch.float32).unsqueeze(2),
                    torch.tensor(u, dtype=torch.float32).unsqueeze(2)).squeeze(2).numpy()
        X.append(xn)
        U.append(u.astype(np.float32))
    X = np.stack(X[:-1], 2).astype(np.float32)   # x_gt[:, :, t] = state at step t
    U = np.stack(U, 2).astype(np.float32)
    sig = np.array([0.02, 0.02, 0.05, 0.05, 0.1])
    Y = (X[:, [0, 1, 3, 4, 5], :] + rng.normal(size=(B, 5, T)) * sig[None, :, None]).astype(np.float32)
    x_mean = X.mean(axis=(0, 2)).reshape(1, 6, 1).astype(np.float32)
    x_std = (X.std(axis=(0, 2)).reshape(1, 6, 1) + 1e-3).astype(np.float32)
    y_mean = Y.mean(axis=(0, 2)).reshape(1, 5, 1).astype(np.float32)
    y_std = (Y.std(axis=(0, 2)).reshape(1, 5, 1) + 1e-3).astype(np.float32)
    t32 = torch.from_numpy
    xm, xs, ym, ys = t32(x_mean), t32(x_std), t32(y_mean), t32(y_std)

    model = KN.KalmanNetNN()
    model.NNBuild(sysm, in_mult_KNet=IN_MULT, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(xm, xs, ym, ys)
    model.load_state_dict({k: torch.tensor(v) for k, v in knet_weights(seed=SEED_W, in_mult=IN_MULT).items()})
    model.eval()
    model.f = sysm.f

    torch.manual_seed(INIT_SEED)                                   # test_prediction.py:172
    x0n_all, xest_all, ades, fdes, profs = [], [], [], [], []
    for i in range(B):
        y, u, x_gt = t32(Y[i]).unsqueeze(0), t32(U[i]).unsqueeze(0), t32(X[i]).unsqueeze(0)
        y_norm = (y - ym) / ys
        x0_norm = (x_gt[:, :, 0] - xm.squeeze(2)) / xs.squeeze(2)
        x0n = (x0_norm + torch.randn_like(x0_norm) * INIT_NOISE_STD).unsqueeze(2)   # :188-191
        x_est = TP.run_full_filter(model, y_norm, u, x0n)
        a, f, pr = [], [], []
        for t in range(T_START, T - H, EVAL_STEP):                 # :199-221
            x_start_real = x_est[:, :, t].unsqueeze(2) * xs + xm
            gt_future = x_gt[:, :, t + 1:t + 1 + H]
            pred = TP.rollout_open_loop(sysm, x_start_real, u, t_start_state=t, H=H)
            assert pred.shape[2] == gt_future.shape[2]
            ade, fde = TP.compute_metrics(pred, gt_future)
            a.append(ade)
            f.append(fde)
            pr.append(TP.get_error_profile(pred, gt_future))
        x0n_all.append(x0n.reshape(6).numpy())
        xest_all.append(x_est.squeeze(0).numpy())
        ades.append(a)
        fdes.append(f)
        profs.append(np.stack(pr))
    np.savez_compressed(
        os.path.join(HERE, "knet_predict.npz"), Ts=Ts, H=H, eval_step=EVAL_STEP, t_start=T_START,
        in_mult=IN_MULT, weight_seed=SEED_W, init_seed=INIT_SEED, init_noise_std=INIT_NOISE_STD,
        limits=np.array([LIMITS[k] for k in sorted(LIMITS)]), limit_names=np.array(sorted(LIMITS)),
        x_mean=x_mean, x_std=x_std, y_mean=y_mean, y_std=y_std, y=Y, u=U, x_gt=X,
        x0n=np.stack(x0n_all), x_est=np.stack(xest_all), ade=np.array(ades, dtype=np.float64),
        fde=np.array(fdes, dtype=np.float64), profile=np.stack(profs).astype(np.float32))
    print("wrote knet_predict.npz", np.array(ades).shape, float(np.mean(ades)), float(np.mean(fdes)))


if __name__ == "__main__":
    main()
