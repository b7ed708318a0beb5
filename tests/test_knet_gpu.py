"""KalmanNet on the GPU (trajectory_generation_amd/knet.py + the HIP ops of include/trajknet.h) vs the
reference's outputs (tests/golden/knet.npz) and the CPU oracle.  float32 throughout, as the reference:
tolerance 2e-4 x (1 + max|ref|) on normalized posteriors (GEMM summation order and single-precision
transcendentals differ from the CPU reference; 20 recurrent steps)."""
import numpy as np
import pytest
import torch

from tests._knet_weights import LIMITS, knet_weights

pytestmark = pytest.mark.gpu
G = np.load("tests/golden/knet.npz")


def build(dev, seed=0, in_mult=5, g=G):
    from trajectory_generation_amd import knet as K
    sysm = K.VehicleModel(float(g["Ts"]), 20, 20, torch.zeros(6, 1))
    sysm.Params.update(LIMITS)
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm, in_mult_KNet=in_mult, out_mult_KNet=40, hidden_dim_gru=128)
    f32 = lambda a: torch.tensor(a, dtype=torch.float32)   # noqa: E731
    model.set_normalization(f32(g["x_mean"]), f32(g["x_std"]), f32(g["y_mean"]), f32(g["y_std"]))
    sd = {k: torch.tensor(v) for k, v in knet_weights(seed=seed, in_mult=in_mult).items()}
    model.load_state_dict(sd, strict=True)
    model.eval()
    return K, sysm, model


def tol(ref):
    return 2e-4 * (1 + np.abs(ref).max())


def test_vehicle_f_h(gpu):
    K, sysm, _ = build(gpu)
    x = torch.tensor(G["phys_x"], dtype=torch.float32, device=gpu).unsqueeze(2)
    u = torch.tensor(G["phys_u"], dtype=torch.float32, device=gpu).unsqueeze(2)
    out = sysm.f(x, u).squeeze(2).cpu().numpy()
    np.testing.assert_allclose(out, G["f_step"], rtol=1e-5, atol=1e-5)
    hh = sysm.h(x).squeeze(2).cpu().numpy()
    np.testing.assert_array_equal(hh, G["phys_x"][:, [0, 1, 3, 4, 5]].astype(np.float32))


def test_missing_limits_raise_like_reference(gpu):
    from trajectory_generation_amd import knet as K
    sysm = K.VehicleModel(0.01, 1, 1, torch.zeros(6, 1))
    x = torch.zeros(2, 6, 1, device=gpu)
    u = torch.zeros(2, 2, 1, device=gpu)
    with pytest.raises(KeyError):
        sysm.f(x, u)


@pytest.mark.parametrize("name", ["knet.npz", "knet_b37_t60_im10.npz"])
def test_sequence_vs_reference(gpu, name):
    g = np.load("tests/golden/" + name)
    _, _, model = build(gpu, seed=int(g["seed"]), in_mult=int(g["in_mult"]), g=g)
    B, T = g["y_norm"].shape[0], g["y_norm"].shape[2]
    y = torch.tensor(g["y_norm"], dtype=torch.float32, device=gpu)
    u = torch.tensor(g["u"], dtype=torch.float32, device=gpu)
    m1x0 = torch.tensor(g["m1x0"], dtype=torch.float32, device=gpu)
    with torch.no_grad():
        model.batch_size = B
        model.init_hidden_KNet()
        model.InitSequence(m1x0, T)
        posts, priors, kgs = [], [], []
        for t in range(T):
            posts.append(model(y[:, :, t:t + 1], u[:, :, t:t + 1]).squeeze(2).cpu().numpy())
            priors.append(model.m1x_prior.squeeze(2).cpu().numpy())
            kgs.append(model.KGain.cpu().numpy())
    post, prior, kg = np.stack(posts, 2), np.stack(priors, 2), np.stack(kgs, 3)
    assert np.abs(prior - g["x_prior"]).max() <= tol(g["x_prior"])
    assert np.abs(kg - g["KG"]).max() <= tol(g["KG"])
    assert np.abs(post - g["x_post"]).max() <= tol(g["x_post"])
    # reference attribute shapes
    assert model.m1x_posterior.shape == (B, 6, 1) and model.KGain.shape == (B, 6, 5)
    assert model.h_Q.shape == (1, B, 128) and model.h_Sigma.shape == (1, B, 128) and model.h_S.shape == (1, B, 128)


def test_graph_runner_matches_eager_and_oracle(gpu):
    from oracle import knet_oracle as KO
    from trajectory_generation_amd.knet import KNetSequenceRunner
    _, sysm, model = build(gpu)
    rng = np.random.default_rng(5)
    B, T = 64, 30
    y = torch.tensor(rng.normal(size=(B, 5, T)), dtype=torch.float32, device=gpu)
    u = torch.tensor(np.stack([rng.uniform(0, 0.5, (B, T)), rng.uniform(-0.3, 0.3, (B, T))], 1), dtype=torch.float32,
                     device=gpu)
    m1x0 = torch.tensor(rng.normal(size=(B, 6, 1)) * 0.5, dtype=torch.float32, device=gpu)
    run = KNetSequenceRunner(model, B)
    eager = run.run(y, u, m1x0, use_graph=False).cpu().numpy()
    g1 = run.run(y, u, m1x0, use_graph=True).cpu().numpy()
    g2 = run.run(y, u, m1x0, use_graph=True).cpu().numpy()    # replay of the captured graph
    np.testing.assert_array_equal(g1, eager)
    np.testing.assert_array_equal(g2, eager)
    p = dict(KO.PARAMS)
    p.update(LIMITS)
    ref = KO.run_sequences(knet_weights(0), p, float(G["Ts"]), y.cpu().numpy(), u.cpu().numpy(), m1x0.cpu().numpy(),
                           G["x_mean"], G["x_std"], G["y_mean"], G["y_std"]).numpy()
    assert np.abs(eager - ref).max() <= 2e-4 * (1 + np.abs(ref).max())


@pytest.mark.parametrize("B,T,groups,in_mult", [(64, 30, 1, 5), (7, 5, 1, 5), (1, 3, 1, 5), (37, 6, 3, 5),
                                                 (64, 30, 1, 10), (37, 6, 3, 10)])
def test_fused_runner_vs_oracle(gpu, B, T, groups, in_mult):
    """Fused step (traj_knet_front_f32 / FC2 GEMMs / traj_knet_back_f32, whole-T graph) vs the CPU oracle,
    ragged batches (B not a multiple of the 4 sequences a workgroup owns) included, for the reference's two
    architectures (in_mult 5: test_vehicle.py / training_prediction.py; 10: training.py / test_prediction.py,
    FC5 60 wide)."""
    from oracle import knet_oracle as KO
    from trajectory_generation_amd.knet import KNetSequenceRunner
    _, sysm, model = build(gpu, seed=1, in_mult=in_mult)
    rng = np.random.default_rng(11 + B)
    y = torch.tensor(rng.normal(size=(B, 5, T)), dtype=torch.float32, device=gpu)
    u = torch.tensor(np.stack([rng.uniform(0, 0.5, (B, T)), rng.uniform(-0.3, 0.3, (B, T))], 1), dtype=torch.float32,
                     device=gpu)
    m1x0 = torch.tensor(rng.normal(size=(B, 6, 1)) * 0.5, dtype=torch.float32, device=gpu)
    run = KNetSequenceRunner(model, B, groups=groups)
    eager = run.run(y, u, m1x0, use_graph=False).cpu().numpy()
    f0 = run.run(y, u, m1x0, use_graph=False, fused=True).cpu().numpy()
    f1 = run.run(y, u, m1x0, fused=True).cpu().numpy()
    f2 = run.run(y, u, m1x0, fused=True).cpu().numpy()       # graph replay
    np.testing.assert_array_equal(f1, f0)
    np.testing.assert_array_equal(f2, f0)
    # back(t) + front(t + 1) merged into one launch == the two launches, bit for bit
    fs = KNetSequenceRunner(model, B, groups=groups, merge=False).run(y, u, m1x0, fused=True).cpu().numpy()
    np.testing.assert_array_equal(fs, f0)
    p = dict(KO.PARAMS)
    p.update(LIMITS)
    ref = KO.run_sequences(knet_weights(1, in_mult=in_mult), p, float(G["Ts"]), y.cpu().numpy(), u.cpu().numpy(),
                           m1x0.cpu().numpy(), G["x_mean"], G["x_std"], G["y_mean"], G["y_std"]).numpy()
    t = 2e-4 * (1 + np.abs(ref).max())
    assert np.abs(f0 - ref).max() <= t
    assert np.abs(f0 - eager).max() <= t


@pytest.mark.parametrize("name", ["knet.npz", "knet_b37_t60_im10.npz"])
def test_fused_runner_vs_reference_goldens(gpu, name):
    """The fused whole-T graph against the reference module's posteriors: B=4 x T=20 (in_mult 5) and a ragged
    B=37 x T=60 batch of the in_mult 10 architecture (tests/golden/gen_knet_golden.py)."""
    from trajectory_generation_amd.knet import KNetSequenceRunner
    g = np.load("tests/golden/" + name)
    _, _, model = build(gpu, seed=int(g["seed"]), in_mult=int(g["in_mult"]), g=g)
    B = g["y_norm"].shape[0]
    y = torch.tensor(g["y_norm"], dtype=torch.float32, device=gpu)
    u = torch.tensor(g["u"], dtype=torch.float32, device=gpu)
    m1x0 = torch.tensor(g["m1x0"], dtype=torch.float32, device=gpu)
    post = KNetSequenceRunner(model, B).run(y, u, m1x0, fused=True).cpu().numpy()
    assert np.abs(post - g["x_post"]).max() <= tol(g["x_post"])


def test_ekf_vs_oracle_and_filters(gpu):
    """EKF baseline (f2): the GPU kernel equals the float64 oracle restatement, and it filters (lower
    state MSE than the raw measurements) on sequences simulated by the reference vehicle model."""
    from oracle import knet_oracle as KO
    from trajectory_generation_amd import knet as K
    p = dict(KO.PARAMS)
    p.update(LIMITS)
    X = G["x_true"].astype(np.float64)            # [4,6,20] simulated with the reference model
    U = G["u"].astype(np.float64)
    rng = np.random.default_rng(3)
    sig = np.sqrt(np.array(K.EKF_R))
    Y = X[:, [0, 1, 3, 4, 5], :] + rng.normal(size=(X.shape[0], 5, X.shape[2])) * sig[None, :, None]
    x0 = X[:, :, 0] + rng.normal(size=(X.shape[0], 6)) * 0.05
    est = K.ekf_run(p, float(G["Ts"]), Y, U, x0).cpu().numpy()
    ref = KO.ekf_run(p, float(G["Ts"]), Y, U, x0, K.EKF_P0, K.EKF_Q, K.EKF_R)
    assert np.abs(est - ref).max() <= 1e-8 * (1 + np.abs(ref).max())
    mse_meas = np.mean((Y - X[:, [0, 1, 3, 4, 5], :]) ** 2)
    mse_ekf = np.mean((est[:, [0, 1, 3, 4, 5], 5:] - X[:, [0, 1, 3, 4, 5], 5:]) ** 2)
    assert mse_ekf < mse_meas


def test_config5_evaluation_pipeline(gpu):
    """knet_eval (configs[4] MSE report): the sequences are the emitter's closed loop plus the reference's
    noise draw (generation_type1.py:312-320), the loss is test_vehicle.py's (checked against a numpy
    restatement), and on those measurements the EKF filters (its loss is below the raw measurements')
    while the seeded-init KalmanNet gives a finite loss."""
    from trajectory_generation_amd import dataset as D
    from trajectory_generation_amd import knet as K
    from trajectory_generation_amd import knet_eval as KE
    B, T, Ts = 16, 40, 0.01
    test = KE.make_sequences(B, T, Ts=Ts, seed=0)
    train = KE.make_sequences(B, T, Ts=Ts, seed=1, id_offset=KE.TRAIN_ID_OFFSET)
    assert test["y"].shape == (B, 5, T) and test["u"].shape == (B, 2, T) and test["x"].shape == (B, 6, T)
    assert (test["status"] <= 1).all()
    noise = np.stack([D.measurement_noise(i, T + 1)[:T] for i in test["ids"]])        # [B,T,6]
    dy = (test["y"] - test["x"][:, [0, 1, 3, 4, 5], :]).cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(dy, noise[:, :, [0, 1, 3, 4, 5]].transpose(0, 2, 1), atol=1e-5)
    xm, xs, ym, ys, lim = KE.normalization(train)
    assert lim["vx_min"] <= float(train["x"][:, 3].min()) and lim["vx_max"] >= float(train["x"][:, 3].max())
    # loss = numpy restatement of test_vehicle.py:15-40
    a = torch.randn(B, 6, T, device=xm.device)
    b = torch.randn(B, 6, T, device=xm.device)
    an, bn = a.cpu().numpy().astype(np.float64), b.cpu().numpy().astype(np.float64)
    xmn, xsn = xm.cpu().numpy().astype(np.float64), xs.cpu().numpy().astype(np.float64)
    dphi = (an * xsn + xmn)[:, 2] - (bn * xsn + xmn)[:, 2]
    ref = 5 / 6 * np.mean((an - bn)[:, [0, 1, 3, 4, 5]] ** 2) + 1 / 6 * np.mean(np.arctan2(np.sin(dphi), np.cos(dphi)) ** 2)
    loss, db = KE.mse_and_db(a, b, xm, xs)
    assert abs(loss - ref) <= 1e-5 * ref and abs(db - 10 * np.log10(ref)) <= 1e-4
    params = dict(K.Params)
    params.update(lim)
    _, ekf_loss, _ = KE.ekf_vs_truth(params, Ts, test, xm, xs, ym, ys)
    y_norm = (test["y"] - ym) / ys
    # raw measurements as the estimate of the measured channels (in the state normalization)
    yx = (test["y"] - xm[:, [0, 1, 3, 4, 5]]) / xs[:, [0, 1, 3, 4, 5]]
    meas_loss = float(((yx - ((test["x"] - xm) / xs)[:, [0, 1, 3, 4, 5], :]) ** 2).mean())
    assert ekf_loss < meas_loss
    torch.manual_seed(0)
    sysm = K.VehicleModel(Ts, T, T, torch.zeros(6, 1))
    sysm.Params.update(lim)
    model = K.KalmanNetNN(xm.device)
    model.NNBuild(sysm)
    model.set_normalization(xm, xs, ym, ys)
    model.eval()
    post = K.KNetSequenceRunner(model, B).run(y_norm.contiguous(), test["u"].contiguous(), KE.hybrid_init(y_norm),
                                              fused=True)
    kl, _ = KE.mse_and_db(post, (test["x"] - xm) / xs, xm, xs)
    assert np.isfinite(kl)
