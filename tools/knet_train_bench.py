"""KalmanNet training-step throughput at the reference's training.py configuration:
in_mult 10, out_mult 40, hidden 128, batch 64, TBPTT chunk 200, AdamW(lr 1e-4, wd 1e-5), composite loss
(alpha 0.8), strategy 'standard'; synthetic data, random-init weights.  T = 200 steps per measured epoch
(one chunk; the reference's T = 1200 is six).  python tools/knet_train_bench.py [B] [T]"""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402
from trajectory_generation_amd import knet_train as KT  # noqa: E402

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
T = int(sys.argv[2]) if len(sys.argv) > 2 else 200
torch.manual_seed(0)
random.seed(0)
sysm = K.VehicleModel(0.01, T, T, torch.zeros(6, 1))
sysm.Params.update(bench.KNET_LIMITS)
model = K.KalmanNetNN(dev)
model.NNBuild(sysm, in_mult_KNet=10, out_mult_KNet=40, hidden_dim_gru=128)
norm = {"x_mean": torch.zeros(1, 6, 1), "x_std": torch.ones(1, 6, 1), "y_mean": torch.zeros(1, 5, 1),
        "y_std": torch.ones(1, 5, 1)}
model.set_normalization(norm["x_mean"], norm["x_std"], norm["y_mean"], norm["y_std"])
x = 0.5 * torch.randn((B, 6, T), device=dev)
y = x[:, [0, 1, 3, 4, 5], :] + 0.05 * torch.randn((B, 5, T), device=dev)
u = 0.2 * torch.randn((B, 2, T), device=dev)
opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
p = dict(strategy="standard", K_TBPTT=200, T=T, m=6, n=5, CompositionLoss=True, alpha=0.8, N_E=B, N_batch=B,
         device=dev)
KT.train_epoch(model, opt, y, u, x, norm, p)     # warm-up (GEMM heuristics, allocator)
torch.cuda.synchronize()
reps = 3
t0 = time.perf_counter()
losses = [KT.train_epoch(model, opt, y, u, x, norm, p)[0] for _ in range(reps)]
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
print(json.dumps({"metric": "KalmanNet training sequence-steps/s (TBPTT, forward + backward + AdamW)",
                  "value": B * T / dt, "unit": "sequence-steps/s", "ms_per_step": 1e3 * dt / T,
                  "config": {"batch": B, "T": T, "K_TBPTT": 200, "in_mult": 10, "out_mult": 40, "hidden": 128,
                             "optimizer": "AdamW(lr 1e-4, wd 1e-5)", "loss": "composite alpha 0.8"},
                  "losses": losses}))
