"""RCCL on the box (diagnostics): the collectives bench.py / dataset.py issue -- barrier, MAX all-reduce of a
float64 scalar, and the dataset gather of one [B, T+1, 9] float64 block per rank (dist.gather, called directly so
that it runs at world size 1 too, where dataset.gather_to_root short-circuits).  Launch with torch.distributed.run;
rank 0 prints one JSON line."""
import datetime
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(B=4096, T=240):
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", timeout=datetime.timedelta(seconds=120), device_id=dev)
    rank, world = dist.get_rank(), dist.get_world_size()
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    blk = torch.randn((B, T + 1, 9), dtype=torch.float64, device=dev, generator=g)
    dist.barrier()
    e = torch.tensor([float(rank) + 0.5], dtype=torch.float64, device=dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    parts = [torch.empty_like(blk) for _ in range(world)] if rank == 0 else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dist.gather(blk, gather_list=parts, dst=0)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ok = True
    if rank == 0:
        ok = torch.equal(parts[0], blk)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "backend": "nccl (RCCL)", "allreduce_max": float(e.item()),
                          "allreduce_ok": float(e.item()) == world - 0.5, "gather_bytes_per_rank": blk.numel() * 8,
                          "gather_s": dt, "gather_rank0_block_equal": bool(ok)}))


if __name__ == "__main__":
    main()
