"""KalmanNet inference throughput (BASELINE.json configs[4]: 1024 sequences x 200 steps, Ts = 0.01):
sequences/s with inputs resident on the GPU, eager vs HIP-graph step.  Development aid; bench.py
reports the same measurement in its JSON line."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tests._knet_weights import LIMITS, knet_weights  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402


def main(B=1024, T=200):
    dev = torch.device("cuda", 0)
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
    run = K.KNetSequenceRunner(model, B)
    for mode in (False, True):
        run.run(y, u, m1x0, use_graph=mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run.run(y, u, m1x0, use_graph=mode)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"graph={mode}: {dt * 1e3:.1f} ms for {B}x{T} -> {B / dt:.0f} seq/s, {dt / T * 1e6:.1f} us/step")


if __name__ == "__main__":
    main()
