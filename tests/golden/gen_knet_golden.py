"""Generate the KalmanNet fixtures in tests/golden/knet.npz from the REFERENCE's own code.

Run in the build container only (reads /root/reference):  python tests/golden/gen_knet_golden.py

Imported read-only from /root/reference/KalmanNet: kalman_net.KalmanNetNN (:5-223) and
vehicle_model.VehicleModel / pt_f_cont / pt_tire_forces (:1-153).  Weights are the deterministic numpy
set of tests/_knet_weights.py (loaded with load_state_dict), eval mode (dropout off), float32 as the
reference runs.  Inputs are synthetic: B=4 sequences of T=20 steps simulated with the reference's own
VehicleModel.f from random initial states and random controls, observed through h with noise.

A second set, knet_b37_t60_im10.npz, covers a ragged batch (B=37, not a multiple of the 4 sequences a fused
workgroup owns), a longer recurrence (T=60) and the in_mult 10 architecture (training.py / test_prediction.py,
FC5 60 wide) with weight seed 2.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests._knet_weights import LIMITS, knet_weights  # noqa: E402

REF = "/root/reference/KalmanNet"


def main(B=4, T=20, in_mult=5, wseed=0, rseed=7, fname="knet.npz"):
    sys.path.insert(0, REF)
    import kalman_net as KN
    import vehicle_model as VM
    torch.set_num_threads(4)
    Ts = 0.01
    rng = np.random.default_rng(rseed)
    params = dict(VM.Params)
    params.update(LIMITS)
    sysm = VM.VehicleModel(Ts, T, T, torch.zeros(6, 1), None, None, None)
    sysm.Params = params

    # physics fixtures
    xp = np.stack([rng.uniform(-2, 30, 64), rng.uniform(-3, 3, 64), rng.uniform(-4, 4, 64),
                   rng.uniform(-0.5, 3.5, 64), rng.uniform(-1.5, 1.5, 64), rng.uniform(-8, 8, 64)], 1)
    up = np.stack([rng.uniform(-1, 1, 64), rng.uniform(-0.6, 0.6, 64)], 1)
    xt = torch.tensor(xp, dtype=torch.float32)
    ut = torch.tensor(up, dtype=torch.float32)
    f_cont = VM.pt_f_cont(xt, ut, params).numpy()
    f_step = sysm.f(xt.unsqueeze(2), ut.unsqueeze(2)).squeeze(2).numpy()

    # synthetic sequences simulated with the reference model
    x = np.stack([rng.uniform(0, 2, B), rng.uniform(-0.5, 0.5, B), rng.uniform(-0.3, 0.3, B),
                  rng.uniform(0.5, 1.5, B), rng.uniform(-0.05, 0.05, B), rng.uniform(-0.5, 0.5, B)], 1)
    X, U = [x], []
    for t in range(T):
        u = np.stack([rng.uniform(0.0, 0.5, B), rng.uniform(-0.3, 0.3, B)], 1)
        xn = sysm.f(torch.tensor(X[-1], dtype=torch.float32).unsqueeze(2),
                    torch.tensor(u, dtype=torch.float32).unsqueeze(2)).squeeze(2).numpy().astype(np.float64)
        X.append(xn)
        U.append(u)
    X = np.stack(X[1:], 2)           # [B,6,T]
    U = np.stack(U, 2)               # [B,2,T]
    sig = np.array([0.02, 0.02, 0.05, 0.05, 0.1])
    Y = X[:, [0, 1, 3, 4, 5], :] + rng.normal(size=(B, 5, T)) * sig[None, :, None]
    x_mean = X.mean(axis=(0, 2)).reshape(1, 6, 1)
    x_std = X.std(axis=(0, 2)).reshape(1, 6, 1) + 1e-3
    y_mean = Y.mean(axis=(0, 2)).reshape(1, 5, 1)
    y_std = Y.std(axis=(0, 2)).reshape(1, 5, 1) + 1e-3
    f32 = lambda a: torch.tensor(a, dtype=torch.float32)   # noqa: E731

    model = KN.KalmanNetNN()
    model.NNBuild(sysm, in_mult_KNet=in_mult, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(f32(x_mean), f32(x_std), f32(y_mean), f32(y_std))
    sd = {k: torch.tensor(v) for k, v in knet_weights(seed=wseed, in_mult=in_mult).items()}
    model.load_state_dict(sd)
    model.eval()
    y_norm = (Y - y_mean) / y_std
    m1x0 = ((X[:, :, 0] - x_mean[:, :, 0]) / x_std[:, :, 0] + 0.1 * rng.normal(size=(B, 6)))[:, :, None]
    post, prior, kg = [], [], []
    with torch.no_grad():
        model.batch_size = B
        model.init_hidden_KNet()
        model.InitSequence(f32(m1x0), T)
        for t in range(T):
            xo = model(f32(y_norm[:, :, t:t + 1]), f32(U[:, :, t:t + 1]))
            post.append(xo.squeeze(2).numpy())
            prior.append(model.m1x_prior.squeeze(2).numpy())
            kg.append(model.KGain.numpy())
    np.savez_compressed(
        os.path.join(HERE, fname), Ts=Ts, seed=wseed, in_mult=in_mult, out_mult=40, hidden=128,
        limits=np.array([LIMITS[k] for k in sorted(LIMITS)]), limit_names=np.array(sorted(LIMITS)),
        phys_x=xp, phys_u=up, pt_f_cont=f_cont, f_step=f_step,
        x_mean=x_mean, x_std=x_std, y_mean=y_mean, y_std=y_std, y_norm=y_norm, u=U, x_true=X, m1x0=m1x0,
        x_post=np.stack(post, 2), x_prior=np.stack(prior, 2), KG=np.stack(kg, 3))
    print("wrote", fname, np.stack(post, 2).shape)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "b37":
        main(B=37, T=60, in_mult=10, wseed=2, rseed=23, fname="knet_b37_t60_im10.npz")
    else:
        main()
