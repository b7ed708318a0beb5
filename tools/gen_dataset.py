"""Closed-loop dataset generation (BASELINE.json configs[3]: 32768 trajectories over the GPUs of one
node, N = 20, dt = 0.05 s, 240 steps), writing the reference's clean / noisy CSV schema.

  python tools/gen_dataset.py --per-gpu 4096 --steps 240 --out vehicle_mpc
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      tools/gen_dataset.py --per-gpu 4096 --steps 240 --out vehicle_mpc

Prints the generation rate (trajectory-steps/s incl. the gather into rank 0, CSV writing excluded) as JSON
on rank 0.  bench.py's dataset leg measures the same with generation and gather timed apart."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-gpu", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=240)
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--dt", type=float, default=0.05)
    ap.add_argument("--kind", default="spline")
    ap.add_argument("--out", default=None, help="CSV prefix (rank 0 writes <out>_clean.csv / <out>_noisy.csv)")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from trajectory_generation_amd import dataset as D
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = D.generate(a.per_gpu, a.steps, N=a.horizon, Ts=a.dt, kind=a.kind, out_prefix=None, dist=dist)
    torch.cuda.synchronize()
    t_gen = time.perf_counter() - t0          # closed loop + gather into rank 0
    if r is not None:                         # rank 0
        X, U, st = r
        t1 = time.perf_counter()
        if a.out:
            import numpy as np
            D.write_csv(a.out, X.cpu().numpy(), U.cpu().numpy(), np.arange(X.shape[0]), a.dt)
        t_csv = time.perf_counter() - t1
        n = X.shape[0] * a.steps
        print(json.dumps({"trajectories": int(X.shape[0]), "steps": a.steps, "n_gpus": world,
                          "traj_steps_per_s": n / t_gen, "generate_s": t_gen, "csv_s": t_csv,
                          "status_hist": torch.bincount(st.reshape(-1).long(), minlength=7).tolist()}))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
