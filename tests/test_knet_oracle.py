"""KalmanNet oracle (oracle/knet_oracle.py) pinned to the reference's own outputs (tests/golden/knet.npz and
knet_b37_t60_im10.npz, made by tests/golden/gen_knet_golden.py from KalmanNet/kalman_net.py + vehicle_model.py).
CPU only."""
import numpy as np
import pytest
import torch

from oracle import knet_oracle as KO
from tests._knet_weights import LIMITS, knet_weights

G = np.load("tests/golden/knet.npz")


def params():
    p = dict(KO.PARAMS)
    p.update(LIMITS)
    return p


def test_weights_fixture_shapes():
    w = knet_weights(seed=int(G["seed"]))
    n = sum(int(np.prod(v.shape)) for v in w.values())
    assert n == 3_191_172   # SURVEY.md App. C (in_mult 5, out_mult 40, hidden 128)


def test_physics_vs_reference():
    x = torch.tensor(G["phys_x"], dtype=torch.float32)
    u = torch.tensor(G["phys_u"], dtype=torch.float32)
    np.testing.assert_allclose(KO.f_cont(x, u, params()).numpy(), G["pt_f_cont"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(KO.f_step(x, u, params(), float(G["Ts"])).numpy(), G["f_step"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("name", ["knet.npz", "knet_b37_t60_im10.npz"])
def test_sequence_vs_reference(name):
    """B=4 x T=20 (in_mult 5) and B=37 x T=60 (in_mult 10, ragged batch) posteriors of the reference module."""
    g = np.load("tests/golden/" + name)
    out = KO.run_sequences(knet_weights(seed=int(g["seed"]), in_mult=int(g["in_mult"])), params(), float(g["Ts"]),
                           g["y_norm"], g["u"], g["m1x0"], g["x_mean"], g["x_std"], g["y_mean"], g["y_std"])
    ref = g["x_post"]
    err = np.abs(out.numpy() - ref).max()
    assert err <= 2e-4 * (1 + np.abs(ref).max()), err
