"""CPU speed of the KalmanNet oracle (oracle/knet_oracle.run_sequences, the bench's cpu_baseline leg)
against the reference's own KalmanNetNN module on the same host and threads.  Build container only
(imports /root/reference/KalmanNet).  Measured 2026-10-16, 8 threads, B=1024, T=10 scaled to 200:
reference module 201 seq/s, oracle 199 seq/s."""
import sys, time, torch, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/reference/KalmanNet')
import kalman_net as KN, vehicle_model as VM
from tests._knet_weights import LIMITS, knet_weights
import oracle.knet_oracle as KO
torch.set_num_threads(8)
B, T = 1024, 10
sysm = VM.VehicleModel(0.01, T, T, torch.zeros(6, 1), torch.eye(6), torch.eye(6), torch.eye(5))
sysm.Params.update(LIMITS)
m = KN.KalmanNetNN(); m.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
m.set_normalization(torch.zeros(1,6,1), torch.ones(1,6,1), torch.zeros(1,5,1), torch.ones(1,5,1))
m.eval(); m.batch_size = B
y = torch.randn(B,5,T); u = 0.2*torch.randn(B,2,T); x0 = 0.5*torch.randn(B,6,1)
with torch.no_grad():
    m.init_hidden_KNet(); m.InitSequence(x0, T)
    t0=time.perf_counter()
    for t in range(T): m(y[:,:,t:t+1], u[:,:,t:t+1])
    dt=time.perf_counter()-t0
print('reference module seq/s (T=200 scaled):', B/(dt*200/T))
w = {k: v.detach() for k, v in m.state_dict().items()}
p = dict(KO.PARAMS); p.update(LIMITS)
z6,o6,z5,o5 = np.zeros((1,6,1)),np.ones((1,6,1)),np.zeros((1,5,1)),np.ones((1,5,1))
t0=time.perf_counter()
KO.run_sequences(w, p, 0.01, y.numpy(), u.numpy(), x0.numpy(), z6,o6,z5,o5)
dt=time.perf_counter()-t0
print('oracle functional seq/s:', B/(dt*200/T))
