"""torch.library registration of the KalmanNet HIP ops (trajectory_generation_amd/knet_ops.py, SURVEY.md 8(b)
torch.ops.trajknet.*): schemas and fake kernels on the CPU (FakeTensorMode, no GPU), and on the GPU the ops
against the module path (kalman_net.py:145-216 through knet.py) and the fused sequence runner -- bit for bit
where the same kernels run, 2e-4 x (1 + max) against the module step (hipBLASLt GEMMs vs the fused kernels)."""
import numpy as np
import pytest
import torch
from torch._subclasses.fake_tensor import FakeTensorMode

from trajectory_generation_amd import knet_ops as KO

B, H = 8, 128
DIMS = [6, 5, 128, 30, 25, 5, 36, 10240]


def test_ops_registered_with_schemas():
    for name in ("prior", "gru_gates", "update", "pack", "step"):
        op = getattr(torch.ops.trajknet, name)
        assert op.default._schema.name == f"trajknet::{name}"
    s = str(torch.ops.trajknet.step.default._schema)
    assert "Tensor[] weights" in s and "float Ts" in s and "Tensor[] norm" in s
    assert len(KO.NET_PTRS) == 27 and KO.PARAM_KEYS[0] == "Cm1"


def test_fake_kernels_propagate_shapes_without_a_gpu():
    with FakeTensorMode():
        f = lambda *s: torch.empty(*s, device="cuda")   # noqa: E731
        ws = [f(4) for _ in KO.NET_PTRS]
        pk = torch.ops.trajknet.pack(ws, DIMS)
        assert pk.dim() == 1 and pk.shape[0] > 0 and pk.device.type == "cuda"
        out = torch.ops.trajknet.step(f(B, 5), f(B, 2), f(B, 6), f(B, H), f(B, H), f(B, H), pk, ws, DIMS,
                                      KO.params_list(), [0.0] * 12, 0.01, [f(6), f(6), f(5), f(5)])
        assert [tuple(o.shape) for o in out] == [(B, 6), (B, H), (B, H), (B, H), (B, 30)]
        pr = torch.ops.trajknet.prior(f(B, 6), f(B, 2), f(B, 5), f(6), f(6), f(5), f(5), None, None,
                                      KO.params_list(), [0.0] * 12, 0.01)
        assert [tuple(o.shape) for o in pr] == [(B, 6), (B, 5), (B, 5)]
        assert torch.ops.trajknet.gru_gates(f(B, 3 * H), f(B, 3 * H), f(B, H)).shape == (B, H)
        assert torch.ops.trajknet.update(f(B, 6), f(B, 30), f(B, 5), f(())).shape == (B, 6)


def test_pack_fake_size_matches_library():
    from trajectory_generation_amd import _lib
    net = _lib.KnetNet()
    for k, v in zip(KO.DIMS, DIMS):
        setattr(net, k, v)
    for k in KO.NET_PTRS:
        setattr(net, k, 16)
    with FakeTensorMode():
        pk = torch.ops.trajknet.pack([torch.empty(4, device="cuda") for _ in KO.NET_PTRS], DIMS)
    assert pk.shape[0] * 4 == _lib.lib().traj_knet_packed_bytes(C_ref(net))


def C_ref(s):
    import ctypes
    return ctypes.byref(s)


# ---------------------------------------------------------------- GPU

def _model(dev, in_mult=5):
    from tests.test_knet_gpu import build
    return build(dev, in_mult=in_mult)


@pytest.mark.gpu
@pytest.mark.parametrize("in_mult", [5, 10])
def test_step_op_matches_fused_runner_and_module(gpu, in_mult):
    from trajectory_generation_amd.knet import KNetSequenceRunner
    K, sysm, model = _model(gpu, in_mult)
    rng = np.random.default_rng(3)
    Bn, T = 37, 3
    y = torch.tensor(rng.normal(size=(Bn, 5, T)), dtype=torch.float32, device=gpu)
    u = torch.tensor(rng.normal(scale=0.3, size=(Bn, 2, T)), dtype=torch.float32, device=gpu)
    m1x0 = torch.tensor(rng.normal(scale=0.5, size=(Bn, 6, 1)), dtype=torch.float32, device=gpu)
    ws, dims = KO.step_weights(model), KO.step_dims(model)
    pk = torch.ops.trajknet.pack(ws, dims)
    norm = list(model._norm_tensors())
    params, limits = KO.params_list(sysm.Params), KO.limits_list(sysm.Params)
    post = m1x0.reshape(Bn, 6)
    hq = hsig = hs = torch.zeros(Bn, 128, device=gpu)
    ops_out = []
    for t in range(T):
        ins = (post, hq, hsig, hs)
        snap = [v.clone() for v in ins]
        post, hq, hsig, hs, KG = torch.ops.trajknet.step(y[:, :, t], u[:, :, t], post, hq, hsig, hs, pk, ws, dims,
                                                         params, limits, sysm.Ts, norm)
        assert all(torch.equal(a, b) for a, b in zip(snap, ins))   # functional: the inputs are untouched
        ops_out.append(post)
    got = torch.stack(ops_out, 2)
    # the fused runner runs the same three kernels per step (unmerged): identical bits
    run = KNetSequenceRunner(model, Bn, merge=False)
    ref = run.run(y, u, m1x0, use_graph=False, fused=True)
    assert torch.equal(got, ref)
    # the module step (hipBLASLt GEMMs + the per-op kernels)
    with torch.no_grad():
        model.batch_size = Bn
        model.init_hidden_KNet()
        model.InitSequence(m1x0, T)
        mod = torch.stack([model(y[:, :, t:t + 1], u[:, :, t:t + 1]).squeeze(2) for t in range(T)], 2)
    assert (got - mod).abs().max().item() <= 2e-4 * (1 + mod.abs().max().item())


@pytest.mark.gpu
def test_prior_gates_update_ops_match_module_kernels(gpu):
    from trajectory_generation_amd import knet as K
    _, sysm, model = _model(gpu)
    rng = np.random.default_rng(4)
    f = lambda *s: torch.tensor(rng.normal(size=s), dtype=torch.float32, device=gpu)   # noqa: E731
    xp, u, y = f(B, 6), f(B, 2), f(B, 5)
    xm, xs, ym, ys = model._norm_tensors()
    a = torch.ops.trajknet.prior(xp, u, y, xm, xs, ym, ys, None, None, KO.params_list(sysm.Params),
                                 KO.limits_list(sysm.Params), sysm.Ts)
    b = K.knet_prior(sysm.Params, sysm.Ts, xp, u, xm, xs, ym, ys, y=y)
    assert all(torch.equal(p, q) for p, q in zip(a, b))
    gi, gh, h = f(B, 3 * H), f(B, 3 * H), f(B, H)
    assert torch.equal(torch.ops.trajknet.gru_gates(gi, gh, h), K._gru_gates(gi, gh, h))
    KG, dy = f(B, 30), f(B, 5)
    got = torch.ops.trajknet.update(xp, KG, dy, model.innov_logit.detach())
    ref = xp + torch.sigmoid(model.innov_logit.detach()) * torch.bmm(KG.reshape(B, 6, 5), dy.reshape(B, 5, 1)).reshape(B, 6)
    assert (got - ref).abs().max().item() <= 1e-5 * (1 + ref.abs().max().item())


@pytest.mark.gpu
def test_op_autograd_matches_module_functions(gpu):
    from trajectory_generation_amd import knet as K
    _, sysm, model = _model(gpu)
    rng = np.random.default_rng(6)
    f = lambda *s: torch.tensor(rng.normal(scale=0.5, size=s), dtype=torch.float32, device=gpu)   # noqa: E731
    xm, xs, ym, ys = model._norm_tensors()
    x0, u, y = f(B, 6), f(B, 2), f(B, 5)
    g = [f(B, 6), f(B, 5), f(B, 5)]
    x1 = x0.clone().requires_grad_(True)
    outs = torch.ops.trajknet.prior(x1, u, y, xm, xs, ym, ys, None, None, KO.params_list(sysm.Params),
                                    KO.limits_list(sysm.Params), sysm.Ts)
    g1, = torch.autograd.grad(outs, [x1], g)
    x2 = x0.clone().requires_grad_(True)
    outs2 = K._KnetPriorFn.apply(x2, u, y, sysm.Params, sysm.Ts, (xm, xs, ym, ys, None, None))
    g2, = torch.autograd.grad(outs2, [x2], g)
    assert torch.equal(g1, g2)
    gi, gh, h = (f(B, 3 * H).requires_grad_(True), f(B, 3 * H).requires_grad_(True), f(B, H).requires_grad_(True))
    go = f(B, H)
    ga = torch.autograd.grad(torch.ops.trajknet.gru_gates(gi, gh, h), [gi, gh, h], [go])
    gb = torch.autograd.grad(K._GruGatesFn.apply(gi, gh, h), [gi, gh, h], [go])
    assert all(torch.equal(p, q) for p, q in zip(ga, gb))
    for op, args in ((torch.ops.trajknet.gru_gates.default, (f(B, 3 * H), f(B, 3 * H), f(B, H))),
                     (torch.ops.trajknet.update.default, (f(B, 6), f(B, 30), f(B, 5),
                                                          torch.tensor(0.3, device=gpu)))):
        torch.library.opcheck(op, args, test_utils=("test_schema", "test_faketensor"))
