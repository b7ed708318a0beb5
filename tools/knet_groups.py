"""Fused KalmanNet sequence throughput vs the number of independent launch chains (graph branches)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402

dev = torch.device("cuda:0")
B, T = int(os.environ.get("KB", 1024)), 200
torch.manual_seed(0)
sysm = K.VehicleModel(0.01, T, T, torch.zeros(6, 1))
sysm.Params.update(bench.KNET_LIMITS)
model = K.KalmanNetNN(dev)
model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
model.eval()
y = torch.randn((B, 5, T), device=dev)
u = 0.2 * torch.randn((B, 2, T), device=dev)
m1x0 = 0.5 * torch.randn((B, 6, 1), device=dev)
ref = None
GS = [int(g) for g in os.environ.get("KG", "1,2,4,8").split(",")]
EAGER = os.environ.get("KEAGER", "0") == "1"
for G in GS:
    run = K.KNetSequenceRunner(model, B, groups=G)
    out = run.run(y, u, m1x0, fused=True, use_graph=not EAGER)
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        run.run(y, u, m1x0, fused=True, use_graph=not EAGER)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    dt = min(ts)
    same = "same" if ref is None or torch.equal(out, ref) else "DIFF %.3g" % (out - ref).abs().max().item()
    ref = out if ref is None else ref
    print(f"groups={G} eager={EAGER}: {B / dt:.0f} seq/s  {1e6 * dt / T:.1f} us/step  {same}", flush=True)
