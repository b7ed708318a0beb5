"""A short fused KalmanNet run for PMC passes (B=1024, T=10, no graph: 3 launches per step)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402

dev = torch.device("cuda:0")
B, T = 1024, 10
torch.manual_seed(0)
sysm = K.VehicleModel(0.01, T, T, torch.zeros(6, 1))
sysm.Params.update(bench.KNET_LIMITS)
model = K.KalmanNetNN(dev)
model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
model.eval()
run = K.KNetSequenceRunner(model, B)
y, u, m1x0 = torch.randn((B, 5, T), device=dev), 0.2 * torch.randn((B, 2, T), device=dev), torch.zeros((B, 6, 1), device=dev)
run.run(y, u, m1x0, fused=True, use_graph=False)
torch.cuda.synchronize()
print("ok")
