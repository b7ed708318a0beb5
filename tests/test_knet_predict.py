"""Sliding-window open-loop prediction evaluation (KalmanNet/test_prediction.py; trajectory_generation_amd/
knet_predict.py + traj_knet_rollout_eval_f32) against the reference's own functions' outputs
(tests/golden/knet_predict.npz, tests/golden/gen_knet_predict_golden.py) and the CPU oracle.

Tolerances: the oracle restates the reference's float32 torch expressions and matches its ADE / FDE /
error profiles to 1e-6 relative; the kernel's single-precision transcendentals differ from the CPU ones
in the last ulp, which 20 to 200 open-loop steps amplify to ~1e-5 relative (bar 1e-4 relative + 1e-6 m);
the full evaluation also inherits the fused filter's 2e-4 x (1 + max) estimate tolerance, so its window
scores are held to 2e-3 relative + 1e-4 m."""
import numpy as np
import pytest
import torch

from tests._knet_weights import LIMITS, knet_weights

G = np.load("tests/golden/knet_predict.npz")
H, STEP, T0, TS = int(G["H"]), int(G["eval_step"]), int(G["t_start"]), float(G["Ts"])


def _params():
    from oracle import knet_oracle as KO
    p = dict(KO.PARAMS)
    p.update(LIMITS)
    return p


# ------------------------------------------------------------------ CPU: oracle pinned to the reference

def test_oracle_window_scores_match_reference():
    from oracle import knet_oracle as KO
    ade, fde, prof = KO.sliding_window_scores(G["x_est"], G["x_mean"], G["x_std"], G["u"], G["x_gt"], _params(),
                                              TS, H, STEP, T0)
    assert ade.shape == G["ade"].shape and prof.shape == G["profile"].shape
    np.testing.assert_allclose(prof.numpy(), G["profile"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(ade.numpy(), G["ade"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(fde.numpy(), G["fde"], rtol=1e-6, atol=1e-7)


def test_oracle_filter_matches_reference_full_filter():
    from oracle import knet_oracle as KO
    w = knet_weights(seed=int(G["weight_seed"]), in_mult=int(G["in_mult"]))
    y_norm = (G["y"] - G["y_mean"]) / G["y_std"]
    out = KO.run_sequences(w, _params(), TS, y_norm, G["u"], G["x0n"][:, :, None], G["x_mean"], G["x_std"],
                           G["y_mean"], G["y_std"]).numpy()
    assert np.abs(out - G["x_est"]).max() <= 2e-5 * (1 + np.abs(G["x_est"]).max())


def test_init_states_reproduce_reference_draws():
    from trajectory_generation_amd import knet_predict as KP
    x0n = KP.init_states(torch.from_numpy(G["x_gt"]), torch.from_numpy(G["x_mean"]), torch.from_numpy(G["x_std"]),
                         "noisy_gt", float(G["init_noise_std"]), int(G["init_seed"]))
    np.testing.assert_array_equal(x0n.squeeze(2).numpy(), G["x0n"])
    with pytest.raises(ValueError):
        KP.init_states(torch.from_numpy(G["x_gt"]), torch.from_numpy(G["x_mean"]), torch.from_numpy(G["x_std"]),
                       "bogus")


def test_window_count_matches_reference_range():
    from trajectory_generation_amd import _lib
    L = _lib.lib()
    for T, h, t0, s in ((1200, 200, 50, 100), (90, 20, 10, 15), (100, 200, 50, 100), (221, 20, 0, 1),
                        (71, 20, 50, 7), (70, 20, 50, 7)):
        assert L.traj_knet_rollout_windows(T, h, t0, s) == len(range(t0, T - h, s))
    assert L.traj_knet_rollout_windows(100, 0, 0, 1) == -1
    assert L.traj_knet_rollout_windows(100, 10, 0, 0) == -1


# ------------------------------------------------------------------ GPU: the kernel and the whole evaluation

def _sys(T):
    from trajectory_generation_amd import knet as K
    sysm = K.VehicleModel(TS, T, T, torch.zeros(6, 1))
    sysm.Params.update(LIMITS)
    return sysm


def _dev(a, gpu):
    return torch.tensor(np.asarray(a), dtype=torch.float32, device=gpu)


@pytest.mark.gpu
def test_window_scores_vs_reference(gpu):
    from trajectory_generation_amd import knet_predict as KP
    T = G["x_gt"].shape[2]
    ade, fde, prof = KP.window_scores(_sys(T), _dev(G["x_est"], gpu), _dev(G["x_mean"], gpu), _dev(G["x_std"], gpu),
                                      _dev(G["u"], gpu), _dev(G["x_gt"], gpu), H, STEP, T0)
    np.testing.assert_allclose(prof.cpu().numpy(), G["profile"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(ade.cpu().numpy(), G["ade"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(fde.cpu().numpy(), G["fde"], rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
def test_sliding_window_eval_vs_reference(gpu):
    from trajectory_generation_amd import knet as K
    from trajectory_generation_amd import knet_predict as KP
    T = G["x_gt"].shape[2]
    sysm = _sys(T)
    model = K.KalmanNetNN(gpu)
    model.NNBuild(sysm, in_mult_KNet=int(G["in_mult"]), out_mult_KNet=40, hidden_dim_gru=128)
    xm, xs, ym, ys = (torch.tensor(G[k]) for k in ("x_mean", "x_std", "y_mean", "y_std"))
    model.set_normalization(xm, xs, ym, ys)
    model.load_state_dict({k: torch.tensor(v) for k, v in
                           knet_weights(seed=int(G["weight_seed"]), in_mult=int(G["in_mult"])).items()})
    model.eval()
    r = KP.sliding_window_eval(model, sysm, torch.tensor(G["y"]), torch.tensor(G["u"]), torch.tensor(G["x_gt"]),
                               xm, xs, ym, ys, H=H, eval_step=STEP, t_start=T0,
                               init_noise_std=float(G["init_noise_std"]), init_seed=int(G["init_seed"]))
    np.testing.assert_array_equal(r["x0n"].squeeze(2).cpu().numpy(), G["x0n"])
    assert np.abs(r["x_est"].cpu().numpy() - G["x_est"]).max() <= 2e-4 * (1 + np.abs(G["x_est"]).max())
    np.testing.assert_allclose(r["ade"].cpu().numpy(), G["ade"], rtol=2e-3, atol=1e-4)
    np.testing.assert_allclose(r["fde"].cpu().numpy(), G["fde"], rtol=2e-3, atol=1e-4)
    assert r["n_windows"] == G["ade"].size
    assert abs(r["ade_mean"] - float(np.mean(G["ade"]))) <= 2e-3 * float(np.mean(G["ade"])) + 1e-4
    assert r["err_time_mean"].shape == (H,)


@pytest.mark.gpu
def test_rollout_open_loop_vs_oracle_and_clipping(gpu):
    from oracle import knet_oracle as KO
    from trajectory_generation_amd import knet_predict as KP
    rng = np.random.default_rng(3)
    B, T = 64, 50
    x0 = np.stack([rng.uniform(0, 20, B), rng.uniform(-3, 3, B), rng.uniform(-1, 1, B), rng.uniform(0.5, 2.5, B),
                   rng.uniform(-0.2, 0.2, B), rng.uniform(-1, 1, B)], 1).astype(np.float32)
    u = np.stack([rng.uniform(0, 0.6, (B, T)), rng.uniform(-0.4, 0.4, (B, T))], 1).astype(np.float32)
    sysm = _sys(T)
    for t0, h in ((10, 30), (35, 30), (0, 50)):   # (35, 30): the reference stops at T (15 steps)
        pred = KP.rollout_open_loop(sysm, _dev(x0, gpu).unsqueeze(2), _dev(u, gpu), t0, h).cpu().numpy()
        ref = KO.rollout_open_loop(torch.from_numpy(x0), torch.from_numpy(u), t0, h, _params(), TS).numpy()
        assert pred.shape == ref.shape == (B, 6, min(h, T - t0))
        np.testing.assert_allclose(pred, ref, rtol=1e-4, atol=1e-5)
    # no step left: the reference returns x0_real
    x0d = _dev(x0, gpu).unsqueeze(2)
    assert KP.rollout_open_loop(sysm, x0d, _dev(u, gpu), T, 5) is x0d


@pytest.mark.gpu
def test_window_scores_full_size_consistency(gpu):
    """test_prediction.py's sizes (H 200, step 100, start 50) on 256 trajectories of 1200 steps: every
    window's profile equals a separate rollout_open_loop of that window scored on the host, and the
    window count is the reference's range()."""
    from trajectory_generation_amd import knet_predict as KP
    rng = np.random.default_rng(9)
    B, T = 256, 1200
    u = np.stack([0.3 + 0.2 * np.sin(0.01 * np.arange(T) + rng.uniform(0, 6, (B, 1))),
                  0.3 * np.sin(0.004 * np.arange(T) + rng.uniform(0, 6, (B, 1)))], 1).astype(np.float32)
    sysm = _sys(T)
    x0 = np.stack([np.zeros(B), np.zeros(B), rng.uniform(-0.3, 0.3, B), rng.uniform(0.8, 1.6, B), np.zeros(B),
                   np.zeros(B)], 1).astype(np.float32)
    xg = KP.rollout_open_loop(sysm, _dev(x0, gpu).unsqueeze(2), _dev(u, gpu), 0, T)        # [B,6,T]
    xg = torch.cat([_dev(x0, gpu).unsqueeze(2), xg[:, :, :-1]], 2)                        # x_gt[:, :, t] = state t
    xm, xs = xg.mean((0, 2)), xg.std((0, 2)) + 1e-3
    x_est = ((xg - xm.reshape(1, 6, 1)) / xs.reshape(1, 6, 1)) + 0.01 * torch.randn_like(xg)
    ade, fde, prof = KP.window_scores(sysm, x_est, xm, xs, _dev(u, gpu), xg)
    W = len(range(KP.T_START_EVAL, T - KP.H_PRED, KP.EVAL_STEP))
    assert ade.shape == (B, W) and prof.shape == (B, W, KP.H_PRED)
    assert torch.isfinite(prof).all()
    for b, w in ((0, 0), (17, 3), (255, W - 1)):
        t = KP.T_START_EVAL + w * KP.EVAL_STEP
        start = (x_est[b:b + 1, :, t] * xs.reshape(1, 6) + xm.reshape(1, 6)).unsqueeze(2)
        pred = KP.rollout_open_loop(sysm, start, _dev(u, gpu)[b:b + 1], t, KP.H_PRED)
        ade_h, fde_h = KP.compute_metrics(pred, xg[b:b + 1, :, t + 1:t + 1 + KP.H_PRED])
        prof_h = KP.get_error_profile(pred, xg[b:b + 1, :, t + 1:t + 1 + KP.H_PRED])
        np.testing.assert_allclose(prof[b, w].cpu().numpy(), prof_h, rtol=1e-6, atol=1e-7)
        assert abs(ade[b, w].item() - ade_h) <= 1e-6 * (1 + abs(ade_h))
        assert abs(fde[b, w].item() - fde_h) <= 1e-6 * (1 + abs(fde_h))


@pytest.mark.gpu
def test_rollout_argument_checks(gpu):
    from trajectory_generation_amd import _lib
    from trajectory_generation_amd import knet_predict as KP
    sysm = _sys(40)
    B, T = 4, 40
    z = lambda *s: torch.zeros(s, dtype=torch.float32, device=gpu)   # noqa: E731
    # a window whose ground truth would run past T is refused
    with pytest.raises(RuntimeError):
        KP._launch(sysm, B, T, 20, 20, 1, 1, z(B, 6, T), (6 * T, T, 1), (z(6), z(6) + 1), z(B, 2, T), z(B, 6, T),
                   z(B), z(B), None, None)
    # no windows: a no-op
    ade, fde, prof = KP.window_scores(sysm, z(B, 6, T), z(6), z(6) + 1, z(B, 2, T), z(B, 6, T), H=50)
    assert ade.shape == (B, 0) and prof.shape == (B, 0, 50)
    assert _lib.TRAJ_E_ARG == -1
