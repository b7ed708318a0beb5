"""FC2 of the fused KalmanNet step (traj_knet_fc2_f32, kalman_net.py:88-95 / :186: Linear(2H, dH) -> ReLU ->
Linear(dH, n m)) in every product mode (traj_knet_set_fc2_mode): the f32 matrix-core form (0) and the three-term
bf16 forms (1, 2 = default), each against a float64 evaluation of the same weights and inputs.  Bar: a float32
GEMM's accuracy, |err| <= 1e-6 x (|b| + |W2b| relu(|W2a| |x2| + |b2a|)) elementwise (the f32 rounding scale of the
two products' absolute sums); the three-term form may not be worse than 2x the f32 form's largest such error, and
its two organizations (every wave splitting the tile, or the tile split once into LDS planes) agree bit for bit."""
import ctypes as C

import numpy as np
import pytest
import torch

from tests._knet_weights import knet_weights

pytestmark = pytest.mark.gpu


def _model(dev, out_mult, seed=3):
    from trajectory_generation_amd import knet as K
    sysm = K.VehicleModel(0.01, 1, 1, torch.zeros(6, 1))
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=out_mult, hidden_dim_gru=128)
    sd = {k: torch.tensor(v) for k, v in knet_weights(seed=seed, out_mult=out_mult).items()}
    model.load_state_dict(sd, strict=True)
    model.eval()
    return K, model


def _fc2(K, model, x2, mode):
    from trajectory_generation_amd import _lib
    L = _lib.lib()
    net = K.net_struct(model)
    B = x2.shape[0]
    ws = torch.full((L.traj_knet_fc2_workspace_bytes(C.byref(net), B) // 4,), float("nan"), device=x2.device)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    prev = L.traj_knet_set_fc2_mode(mode)
    try:
        _lib.check(L.traj_knet_fc2_f32(C.byref(net), B, C.c_void_p(x2.data_ptr()), C.c_void_p(ws.data_ptr()),
                                       ws.numel() * 4, st), "traj_knet_fc2_f32")
    finally:
        L.traj_knet_set_fc2_mode(prev)
    torch.cuda.synchronize()
    nm = model.n * model.m
    part = ws.reshape(-1, B, 32).double().cpu().numpy()[:, :, :nm]
    b2b = model.FC2[2].bias.detach().double().cpu().numpy()
    return b2b[None, :] + part.sum(0)


@pytest.mark.parametrize("out_mult,B", [(40, 1024), (40, 37), (5, 70), (2, 64)])
def test_fc2_modes_vs_float64(gpu, out_mult, B):
    """out_mult 40: the reference's FC2 (10240 hidden units, slabs of 320 on the XCD-grouped grid); 5: 1280 (slabs of
    320, plain grid); 2: 512 (slabs of 256); ragged B (rows past B duplicated, never stored)."""
    K, model = _model(gpu, out_mult)
    rng = np.random.default_rng(out_mult + B)
    x2h = np.maximum(rng.normal(size=(B, 256)), 0.0).astype(np.float32) * 2.0
    x2h[:, ::3] = rng.normal(size=(B, x2h[:, ::3].shape[1])).astype(np.float32)   # signed entries as well
    x2 = torch.tensor(x2h, device=gpu)
    Wa = model.FC2[0].weight.detach().double().cpu().numpy()
    ba = model.FC2[0].bias.detach().double().cpu().numpy()
    Wb = model.FC2[2].weight.detach().double().cpu().numpy()
    bb = model.FC2[2].bias.detach().double().cpu().numpy()
    xd = x2h.astype(np.float64)
    hid = np.maximum(xd @ Wa.T + ba, 0.0)
    ref = hid @ Wb.T + bb
    scale = np.abs(bb) + np.maximum(np.abs(xd) @ np.abs(Wa).T + np.abs(ba), 0.0) @ np.abs(Wb).T
    errs, outs = {}, {}
    for mode in (0, 1, 2):
        out = _fc2(K, model, x2, mode)
        assert np.isfinite(out).all()
        rel = np.abs(out - ref) / scale
        assert rel.max() <= 1e-6, (mode, rel.max())
        errs[mode], outs[mode] = rel.max(), out
    assert errs[2] <= 2.0 * errs[0] + 1e-7, errs
    np.testing.assert_array_equal(outs[1], outs[2])


def test_fc2_mode_switch(gpu):
    from trajectory_generation_amd import _lib
    L = _lib.lib()
    assert L.traj_knet_set_fc2_mode(3) == -1 and L.traj_knet_set_fc2_mode(-1) == -1
    prev = L.traj_knet_set_fc2_mode(0)
    assert prev == 2   # the default: the three-term form, tile split once per workgroup
    assert L.traj_knet_set_fc2_mode(prev) == 0
