"""FC2 alone for PMC passes: `python tools/knet_fc2_pmc.py MODE [REPS]` runs traj_knet_fc2_f32 at
configs[4]'s B = 1024 REPS times (default 20) in FC2 mode MODE (traj_knet_set_fc2_mode).  Run under
`rocprofv3 --pmc ...` (one pass per counter group); development aid."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tests._knet_weights import knet_weights  # noqa: E402
from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import knet as K  # noqa: E402


def main(mode, reps=20, B=1024):
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    sysm = K.VehicleModel(0.01, 1, 1, torch.zeros(6, 1))
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm)
    model.load_state_dict({k: torch.tensor(v) for k, v in knet_weights(0).items()})
    model.eval()
    net = K.net_struct(model)
    x2 = torch.relu(torch.randn(B, 256, device=dev))
    ws = torch.empty(L.traj_knet_fc2_workspace_bytes(C.byref(net), B) // 4, device=dev)
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    L.traj_knet_set_fc2_mode(mode)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for it in range(reps):
        if it == reps // 2:
            e0.record()
        rc = L.traj_knet_fc2_f32(C.byref(net), B, C.c_void_p(x2.data_ptr()), C.c_void_p(ws.data_ptr()),
                                 ws.numel() * 4, st)
        _lib.check(rc, "fc2")
    e1.record()
    torch.cuda.synchronize()
    print(f"fc2 mode {mode}: {e0.elapsed_time(e1) * 1e3 / (reps - reps // 2):.2f} us per launch "
          f"({os.environ.get('TRAJMPC_LIB', 'in-tree')})")


if __name__ == "__main__":
    main(int(sys.argv[1]), int(sys.argv[2]) if len(sys.argv) > 2 else 20)
