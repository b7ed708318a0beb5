"""Fused KalmanNet step vs batch size (rocprofv3 --kernel-trace groups the kernels by grid size):
python tools/knet_scaling.py  [B values]."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402

dev = torch.device("cuda:0")
T = 50
torch.manual_seed(0)
sysm = K.VehicleModel(0.01, T, T, torch.zeros(6, 1))
sysm.Params.update(bench.KNET_LIMITS)
model = K.KalmanNetNN(dev)
model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
model.eval()
for B in [int(a) for a in sys.argv[1:]] or [256, 512, 1024, 2048, 4096]:
    y = torch.randn((B, 5, T), device=dev)
    u = 0.2 * torch.randn((B, 2, T), device=dev)
    m1x0 = 0.5 * torch.randn((B, 6, 1), device=dev)
    run = K.KNetSequenceRunner(model, B)
    run.run(y, u, m1x0, fused=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.run(y, u, m1x0, fused=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"B={B}: {B / dt * T / 200:.0f} seq/s (T=200 equiv)  {1e6 * dt / T:.1f} us/step", flush=True)
