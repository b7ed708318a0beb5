"""bench.py's multi-rank path on CPU (no GPU): bench_run's distributed branch end to end at world sizes 2 and 4
over gloo -- barriers, the MAX all-reduce of the elapsed time, the dataset leg's gather into rank 0, the
record on rank 0 only -- with a CPU stand-in for the device side; and the launcher's failure handling (a
worker that dies takes its siblings down, the parent exits with its status)."""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


class CpuOps:
    """Same interface as bench.GpuOps; deterministic arithmetic instead of the MPC (the test checks the
    orchestration, not the solver)."""

    def __init__(self, local):
        self.dev = torch.device("cpu")

    def sync(self):
        pass

    def setup(self, w, B, N, Ts, T, polish_mode, warm_start=1):
        x = torch.as_tensor(w["x0"]).clone()
        s = dict(x=x, hx=torch.zeros((B, T + 1, 6), dtype=torch.float64), hu=torch.zeros((B, T, 2), dtype=torch.float64),
                 st=torch.zeros((T, B), dtype=torch.int32), it=torch.zeros((T, B), dtype=torch.int32), kmax=11,
                 cfg=type("Cfg", (), {"warm_start": warm_start})())
        s["hx"][:, 0] = x
        return s

    def run(self, s, t0, steps, fused):
        for t in range(t0, t0 + steps):
            s["x"] += 0.01
            s["hx"][:, t + 1] = s["x"]
            s["st"][t] = 0
            s["it"][t] = 25 if s["cfg"].warm_start else 50
        time.sleep(0.06 if os.environ.get("RANK") == "1" else 0.01)   # rank 1 is the slow one

    def kernel_timing(self, steps):
        pass

    def kernel_times(self):
        return {"rollout_kernel": 0.0, "jac_kernel": 0.0, "order_kernel": 0.0, "solve_kernel": 1.0}

    def closed_loop(self, w, T, N, Ts, polish_mode):
        x0 = torch.as_tensor(w["x0"])
        B = x0.shape[0]
        X = x0[:, None, :] + 0.01 * torch.arange(T + 1, dtype=torch.float64)[None, :, None]
        U = torch.zeros((B, T, 2), dtype=torch.float64)
        return X, U, torch.zeros((T, B), dtype=torch.int32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, q, csv_dir, world=2):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import bench
    out = bench.main(["--gpus", str(world), "--steps", "3", "--warmup", "1", "--batch", "4", "--dataset-steps", "5",
                      "--no-cpu", "--no-knet", "--dist-timeout", "120", "--dataset-csv", csv_dir],
                     ops_factory=CpuOps, backend="gloo")
    q.put((rank, out))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_run_multi_rank_gloo(tmp_path, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q, str(tmp_path), world)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(got[r] is None for r in range(1, world))     # one record, from rank 0
    out = got[0]
    G = 4 * world
    assert out["n_gpus"] == world and out["config"]["global_batch"] == G and out["scaling"] == "weak"
    assert out["value"] == pytest.approx(G * 3 / (out["ms_per_step"] * 3 / 1e3))   # whole-job steps / max elapsed
    assert out["ms_per_step"] >= 18.0                       # the MAX over ranks: rank 1's 60 ms for 3 steps
    assert out["cold"]["iters_mean"] == 50.0 and out["solver_stats"]["iters_mean"] == 25.0
    ds = out["dataset"]
    assert ds["trajectories"] == G and ds["steps"] == 5 and ds["gather_bytes"] == G * 6 * 9 * 8
    assert ds["status_hist"][0] == G * 5 and ds["failed_trajectories"] == 0
    # the gathered files on rank 0 and one shard per rank (ids 4r .. 4r+3), each with its status sidecar
    assert ds["csv_s"] is not None and ds["csv_shards_s"] is not None
    one = open(tmp_path / "vehicle_mpc_clean.csv").read().splitlines()
    sh = [open(tmp_path / f"vehicle_mpc_rank{r}_clean.csv").read().splitlines() for r in range(world)]
    assert sum((x[1:] for x in sh), []) == one[1:] and len(one) == 1 + G * 6
    for r in range(world):
        assert len(open(tmp_path / f"vehicle_mpc_rank{r}_status.csv").read().splitlines()) == 5


def test_spawned_worker_failure_stops_the_siblings():
    """_spawn_workers: worker 1 exits 3 at once, worker 0 would sleep a minute -- the parent terminates it and
    exits 3 within seconds (a rank that dies before the rendezvous must not leave the others blocked)."""
    import bench
    script = ("import os, sys, time\n"
              "if os.environ['RANK'] == '1': sys.exit(3)\n"
              "time.sleep(60)\n")
    t0 = time.time()
    with pytest.raises(SystemExit) as e:
        bench._spawn_workers(2, poll_s=0.05, grace_s=5.0, cmd=[sys.executable, "-c", script])
    assert e.value.code == 3
    assert time.time() - t0 < 20


def test_bench_world1_config3_host_io_and_profile_reasons(tmp_path, monkeypatch):
    """The one-GPU line's extra objects with the CPU stand-in: config3 (configs[2]: N = 40 mixed, the same timed-region
    contract) with its own roofline, host_io (H2D + run + D2H), the timed-region note, and a profile that does not
    describe the launch is rejected with the reason recorded instead of a silent null."""
    import json
    import bench
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    bad = tmp_path / "sq.json"
    bad.write_text(json.dumps({"batch": 4, "horizon": 20, "f64_flop_issued_per_step": 1.0, "valu_insts_per_step": 1.0}))
    out = bench.main(["--steps", "3", "--warmup", "1", "--batch", "4", "--dataset-steps", "0", "--no-cpu", "--no-knet",
                      "--no-config1", "--config3-issue-json", str(bad), "--issue-json", str(bad),
                      "--traffic-json", str(tmp_path / "none.json")], ops_factory=CpuOps, backend="gloo")
    assert out["n_gpus"] == 1 and "H2D / D2H excluded" in out["config"]["timed_region"]
    assert out["roofline"]["issue"] is not None and out["roofline"]["issue"]["source"].endswith("sq.json")
    assert "not found" in out["roofline"]["traffic_rejected"]
    c3 = out["config3"]
    assert c3["config"]["horizon"] == 40 and c3["value"] > 0 and c3["roofline"]["kernel"].startswith("solve_split_kernel<40,true,true>")
    assert c3["roofline"]["issue"] is None and "horizon = 20, this launch has 40" in c3["roofline"]["issue_rejected"]
    hio = out["host_io"]
    assert hio["value"] > 0 and hio["steps"] == 4 and hio["d2h_bytes"] == 4 * 5 * 6 * 8 + 4 * 4 * 2 * 8 + 2 * 4 * 4 * 4
