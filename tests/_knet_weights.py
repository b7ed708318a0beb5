"""Deterministic KalmanNet weights for the parity fixtures (numpy RNG, so they do not depend on the
torch version's default initialisation).  Shapes follow KalmanNet/kalman_net.py:26-113 (NNBuild)."""
import numpy as np

M, N_OBS = 6, 5


def knet_shapes(in_mult=5, out_mult=40, hidden=128, m=M, n=N_OBS):
    fc5 = m * in_mult
    fc1 = n * n
    d_in_s = fc1 + n
    d_in_fc2 = 2 * hidden
    d_hid_fc2 = d_in_fc2 * out_mult
    fc2_out = n * m
    fc3_out = m * m
    sh = {"innov_logit": ()}
    sh["FC5.0.weight"], sh["FC5.0.bias"] = (fc5, m), (fc5,)
    for name, din in (("GRU_Q", fc5), ("GRU_Sigma", hidden), ("GRU_S", d_in_s)):
        sh[f"{name}.weight_ih_l0"] = (3 * hidden, din)
        sh[f"{name}.weight_hh_l0"] = (3 * hidden, hidden)
        sh[f"{name}.bias_ih_l0"] = (3 * hidden,)
        sh[f"{name}.bias_hh_l0"] = (3 * hidden,)
    sh["FC1.0.weight"], sh["FC1.0.bias"] = (fc1, hidden), (fc1,)
    sh["FC7.0.weight"], sh["FC7.0.bias"] = (n, n), (n,)
    sh["FC2.0.weight"], sh["FC2.0.bias"] = (d_hid_fc2, d_in_fc2), (d_hid_fc2,)
    sh["FC2.2.weight"], sh["FC2.2.bias"] = (fc2_out, d_hid_fc2), (fc2_out,)
    sh["FC3.0.weight"], sh["FC3.0.bias"] = (fc3_out, hidden + fc2_out), (fc3_out,)
    sh["FC4.0.weight"], sh["FC4.0.bias"] = (hidden, hidden + fc3_out), (hidden,)
    return sh


def knet_weights(seed=0, in_mult=5, out_mult=40, hidden=128, innov_logit=0.3):
    """float32 arrays keyed like the reference state_dict: U(-1/sqrt(fan_in), 1/sqrt(fan_in))."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, shp in knet_shapes(in_mult, out_mult, hidden).items():
        if k == "innov_logit":
            out[k] = np.array(innov_logit, dtype=np.float32)
            continue
        if k.startswith("GRU"):
            fan = shp[1] if len(shp) == 2 else hidden   # torch GRU: U(-1/sqrt(hidden), 1/sqrt(hidden))
            bound = 1.0 / np.sqrt(hidden)
        else:
            fan = shp[1] if len(shp) == 2 else None
            bound = 1.0 / np.sqrt(fan) if fan else 0.05
        out[k] = rng.uniform(-bound, bound, size=shp).astype(np.float32)
    return out


# clamp limits injected into the vehicle Params by the caller (vehicle_model.py:54-57,125-131)
LIMITS = {"x_min": -5.0, "x_max": 40.0, "y_min": -6.0, "y_max": 6.0, "phi_min": -3.2, "phi_max": 3.2,
          "vx_min": 0.0, "vx_max": 3.0, "vy_min": -1.0, "vy_max": 1.0, "omega_min": -6.0, "omega_max": 6.0}
