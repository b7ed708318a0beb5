"""Bit-level comparison of the step entry point between library builds (diagnostics only).

  python tools/split_bitcmp.py save OUT.npz [N]      (the library named by TRAJMPC_LIB, or the in-tree one)
  python tools/split_bitcmp.py cmp A.npz B.npz ...

save: traj_mpc_step_batch on 512 random parabola windows (dt 0.05) at N (default 40), every output saved.
cmp: per output, the number of instances whose values differ in any bit, against the first file."""
import sys

import numpy as np


def save(out, N):
    import torch
    sys.path.insert(0, ".")
    from trajectory_generation_amd import batch as TB
    from tools.horizon_tiers import instances
    x0, up, pr, vr = instances(512, N, 0.05)
    d = [torch.as_tensor(a, device="cuda") for a in (x0, up, pr, vr)]
    o = TB.mpc_step_batch(*d, TB.config_struct(N=N, Ts=0.05))
    np.savez(out, **{k: v.cpu().numpy() for k, v in o.items()})


def cmp(files):
    ref = np.load(files[0])
    for f in files[1:]:
        o = np.load(f)
        res = {}
        for k in ref.files:
            a, b = ref[k].reshape(len(ref[k]), -1), o[k].reshape(len(o[k]), -1)
            diff = ~((a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)).all(axis=1)
            res[k] = int(diff.sum())
        print(f, res, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "save":
        save(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
    else:
        cmp(sys.argv[2:])
