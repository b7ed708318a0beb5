"""FC2 product modes (traj_knet_set_fc2_mode) at configs[4] (1024 sequences x 200 steps): the fused runner's
sequences/s and one FC2 launch's time (HIP events over 50 launches) per mode, and the largest posterior
difference between the modes.  Development aid; prints one JSON object."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests._knet_weights import LIMITS, knet_weights  # noqa: E402
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402


def main(B=1024, T=200, reps=5):
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    sysm = K.VehicleModel(0.01, T, T, torch.zeros(6, 1))
    sysm.Params.update(LIMITS)
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm)
    model.load_state_dict({k: torch.tensor(v) for k, v in knet_weights(0).items()})
    model.set_normalization(torch.zeros(1, 6, 1), torch.ones(1, 6, 1), torch.zeros(1, 5, 1), torch.ones(1, 5, 1))
    model.eval()
    rng = np.random.default_rng(0)
    y = torch.tensor(rng.normal(size=(B, 5, T)), dtype=torch.float32, device=dev)
    u = torch.tensor(rng.normal(size=(B, 2, T)) * 0.2, dtype=torch.float32, device=dev)
    m1x0 = torch.zeros(B, 6, 1, device=dev)
    net = K.net_struct(model)
    x2 = torch.relu(torch.randn(B, 256, device=dev))
    ws = torch.empty(L.traj_knet_fc2_workspace_bytes(C.byref(net), B) // 4, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def fc2():
        return L.traj_knet_fc2_f32(C.byref(net), B, C.c_void_p(x2.data_ptr()), C.c_void_p(ws.data_ptr()),
                                   ws.numel() * 4, st)

    res = {}
    outs = {}
    for mode in (0, 1, 2, 0, 1, 2):
        L.traj_knet_set_fc2_mode(mode)
        run = K.KNetSequenceRunner(model, B)
        out = run.run(y, u, m1x0, fused=True)   # capture + warm
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            out = run.run(y, u, m1x0, fused=True)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        outs[mode] = out.cpu().numpy()
        key = f"mode{mode}"
        r = res.setdefault(key, {"seq_per_s": [], "step_us": [], "fc2_us": []})
        r["seq_per_s"].append(round(B / best, 1))
        r["step_us"].append(round(best / T * 1e6, 2))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            fc2()
        e0.record()
        for _ in range(50):
            fc2()
        e1.record()
        torch.cuda.synchronize()
        r["fc2_us"].append(round(e0.elapsed_time(e1) * 1e3 / 50, 2))
    L.traj_knet_set_fc2_mode(2)
    res["max_abs_diff_posteriors"] = float(np.abs(outs[0] - outs[2]).max())
    res["modes_1_2_identical"] = bool(np.array_equal(outs[1], outs[2]))
    res["max_abs_posterior"] = float(np.abs(outs[0]).max())
    flop = B * 2 * (256 * 10240 + 10240 * 30)
    res["fc2_flop"] = flop
    print(json.dumps(res))


if __name__ == "__main__":
    main()
