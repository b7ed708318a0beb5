"""Dataset emitter schema/noise (generation_traj/generation_type1.py:139-158, :295-339) and the
multi-process gather (gloo, world size 2, CPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from trajectory_generation_amd import dataset as D


def test_noise_is_the_reference_draw():
    # generation_type1.py:312-320: default_rng(12345 + i), one normal(0, std, N) per channel
    for tid in (0, 7, 4095):
        rng = np.random.default_rng(12345 + tid)
        ref = np.column_stack([rng.normal(0, 0.05, 241), rng.normal(0, 0.05, 241), rng.normal(0, 0.003, 241),
                               rng.normal(0, 0.010, 241), rng.normal(0, 0.003, 241), rng.normal(0, 0.030, 241)])
        np.testing.assert_array_equal(D.measurement_noise(tid, 241), ref)


def test_frames_schema():
    B, T = 3, 5
    rng = np.random.default_rng(0)
    X = rng.normal(size=(B, T + 1, 6))
    U = rng.normal(size=(B, T, 2))
    clean, noisy = D.frames(X, U, [10, 11, 12], 0.05)
    assert list(clean.columns) == ["t", "X", "Y", "phi", "vx", "vy", "omega", "d", "delta", "trajectory_id"]
    assert list(noisy.columns) == ["t", "X", "Y", "vx", "vy", "omega", "d", "delta", "trajectory_id"]
    assert len(clean) == B * (T + 1) and len(noisy) == B * (T + 1)
    last = clean.groupby("trajectory_id").tail(1)
    assert last["d"].isna().all() and last["delta"].isna().all()
    assert clean["d"].isna().sum() == B
    np.testing.assert_array_equal(clean["X"].to_numpy().reshape(B, T + 1), X[:, :, 0])
    np.testing.assert_allclose(noisy["X"].to_numpy().reshape(B, T + 1) - X[:, :, 0],
                               np.stack([D.measurement_noise(i, T + 1)[:, 0] for i in (10, 11, 12)]))
    np.testing.assert_allclose(clean["t"].to_numpy()[: T + 1], np.arange(T + 1) * 0.05)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_closed_loop(w, T, cfg):
    """CPU stand-in for one rank's closed loop: histories that encode the trajectory id and the step."""
    ids = np.asarray(w["ids"], dtype=np.float64)
    B = len(ids)
    X = torch.tensor(ids[:, None, None] + 0.01 * np.arange(T + 1)[None, :, None] + w["x0"][:, None, :] * 0.0)
    X[:, 0] = torch.tensor(w["x0"])
    U = torch.tensor(-ids[:, None, None] + np.zeros((1, T, 2)))
    st = torch.tensor((ids[None, :].astype(np.int64) + np.arange(T)[:, None]) % 7, dtype=torch.int32)
    return dict(X=X, U=U, status=st)


def _worker(rank, world, port, q, out_prefix, shards=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, T = 4, 6
    r = D.generate(B, T, N=20, Ts=0.05, kind="spline", seed=3, out_prefix=out_prefix, dist=dist,
                   closed_loop=_fake_closed_loop, shards=shards, drop_failed=False)
    if shards:
        q.put((rank, r[0].numpy(), r[1].numpy(), r[2].numpy()))
    elif rank == 0:
        X, U, st = r
        q.put((X.numpy(), U.numpy(), st.numpy()))
    else:
        q.put(r)
    dist.barrier()
    dist.destroy_process_group()


def test_generate_two_ranks_gloo(tmp_path):
    """dataset.generate at world size 2 (gloo): rank r runs ids [r B, (r+1) B) (the workload's own id
    offset; merge_datasets.py:41-47 offsets ids the same way), the packed histories and statuses reach rank 0 only,
    in id order, and rank 0 writes the CSVs with the global trajectory ids."""
    from trajectory_generation_amd.workload import make_workload
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    prefix = str(tmp_path / "ds")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, prefix)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sum(g is None for g in got) == 1          # rank 1 receives nothing
    gX, gU, st = next(g for g in got if g is not None)
    assert gX.shape == (8, 7, 6) and gU.shape == (8, 6, 2) and st.shape == (6, 8)
    np.testing.assert_array_equal(gX[:, 1, 0], np.arange(8) + 0.01)   # rank order == global id order
    np.testing.assert_array_equal(gU[:, 0, 0], -np.arange(8))
    np.testing.assert_array_equal(st, (np.arange(8)[None, :] + np.arange(6)[:, None]) % 7)
    # step 0 = each id's own initial state: rank 1's share is ids 4..7 of the same seeded workload
    w = make_workload(8, 20, 0.05, kind="spline", seed=3)
    np.testing.assert_array_equal(gX[:, 0, :], w["x0"])
    import pandas as pd
    clean = pd.read_csv(prefix + "_clean.csv")
    noisy = pd.read_csv(prefix + "_noisy.csv")
    assert sorted(clean["trajectory_id"].unique()) == list(range(8))
    assert len(clean) == 8 * 7 and len(noisy) == 8 * 7
    np.testing.assert_allclose(clean["X"].to_numpy().reshape(8, 7), gX[:, :, 0], rtol=0, atol=1e-12)


def test_generate_two_ranks_per_rank_shards_gloo(tmp_path):
    """shards=True (SURVEY.md 8(e)'s per-rank alternative): no gather, each rank writes its own CSV shard and
    status sidecar with the global ids; the shards' bodies concatenated in rank order are byte for byte the
    single gathered file's body."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    prefix = str(tmp_path / "sh")
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, prefix, True)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted([q.get(timeout=120) for _ in range(2)], key=lambda g: g[0])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    X = np.concatenate([g[1] for g in got])
    U = np.concatenate([g[2] for g in got])
    st = np.concatenate([g[3] for g in got], axis=1)
    D.write_csv(str(tmp_path / "one"), X, U, np.arange(8), 0.05)
    D.write_status_csv(str(tmp_path / "one"), st, np.arange(8))
    for part in ("clean", "noisy", "status"):
        one = open(tmp_path / f"one_{part}.csv").read().splitlines()
        shards = [open(f"{prefix}_rank{r}_{part}.csv").read().splitlines() for r in range(2)]
        assert shards[0][0] == shards[1][0] == one[0]
        assert shards[0][1:] + shards[1][1:] == one[1:]


def _status_closed_loop(w, T, cfg):
    """Stand-in with chosen statuses: trajectory 2 fails at step 1 (solver error), 4 at step 3 (iteration
    limit, status 2); everything else optimal / optimal_inaccurate."""
    r = _fake_closed_loop(w, T, cfg)
    st = torch.zeros((T, len(w["ids"])), dtype=torch.int32)
    st[0, 1] = 1
    st[1, 2] = 6
    st[3, 4] = 2
    r["status"] = st
    return r


def test_status_sidecar_and_failed_trajectory_filter(tmp_path):
    """The reference's CSV schema carries no status: generate writes {prefix}_status.csv beside it (worst
    status, failed-step count, first failed step per trajectory) and, with drop_failed, leaves out the
    trajectories with a failed step and re-indexes the rest 0..n-1 (the ids data_loader.py reads), each
    keeping the noise draw of its generation id."""
    import pandas as pd
    B, T = 6, 4
    p1 = str(tmp_path / "all")
    X, U, st = D.generate(B, T, N=20, Ts=0.05, seed=3, out_prefix=p1, closed_loop=_status_closed_loop,
                          drop_failed=False)
    sc = pd.read_csv(p1 + "_status.csv")
    assert list(sc.columns) == ["trajectory_id", "source_id", "worst_status", "n_failed_steps", "first_failed_step"]
    assert sc["worst_status"].tolist() == [0, 1, 6, 0, 2, 0]
    assert sc["n_failed_steps"].tolist() == [0, 0, 1, 0, 1, 0]
    assert sc["first_failed_step"].tolist() == [-1, -1, 1, -1, 3, -1]
    assert list(pd.read_csv(p1 + "_clean.csv").columns) == D.CLEAN_COLUMNS   # schema unchanged
    p2 = str(tmp_path / "ok")
    p0 = str(tmp_path / "dflt")
    D.generate(B, T, N=20, Ts=0.05, seed=3, out_prefix=p0, closed_loop=_status_closed_loop)   # default: all written
    assert pd.read_csv(p0 + "_status.csv")["trajectory_id"].tolist() == list(range(B))
    assert (tmp_path / "dflt_clean.csv").read_bytes() == (tmp_path / "all_clean.csv").read_bytes()
    with pytest.warns(UserWarning, match="left out 2 of 6"):
        D.generate(B, T, N=20, Ts=0.05, seed=3, out_prefix=p2, closed_loop=_status_closed_loop, drop_failed=True)
    sc2 = pd.read_csv(p2 + "_status.csv")
    assert sc2["trajectory_id"].tolist() == [0, 1, 2, 3] and sc2["source_id"].tolist() == [0, 1, 3, 5]
    assert (sc2["n_failed_steps"] == 0).all()
    clean = pd.read_csv(p2 + "_clean.csv")
    noisy = pd.read_csv(p2 + "_noisy.csv")
    assert sorted(clean["trajectory_id"].unique()) == [0, 1, 2, 3]
    Xn = X.numpy()
    keep = [0, 1, 3, 5]
    np.testing.assert_array_equal(clean["X"].to_numpy().reshape(4, T + 1), Xn[keep, :, 0])
    noise = np.stack([D.measurement_noise(i, T + 1)[:, 0] for i in keep])
    np.testing.assert_allclose(noisy["X"].to_numpy().reshape(4, T + 1), Xn[keep, :, 0] + noise, rtol=0, atol=1e-12)
    res = D.load_vehicle_dataset(p2 + "_noisy.csv", p2 + "_clean.csv", T_steps=T + 1, train_split=0.5, val_split=0.25)
    assert res is not None and sum(part[0].shape[0] for part in res) == 4
    with pytest.raises(ValueError):
        D.generate(B, T, out_prefix=p2, closed_loop=_status_closed_loop, drop_failed=True, shards=True)


def test_pack_unpack_history():
    B, T = 3, 5
    X = torch.randn(B, T + 1, 6, dtype=torch.float64)
    U = torch.randn(B, T, 2, dtype=torch.float64)
    st = torch.randint(0, 7, (T, B), dtype=torch.int32)
    X2, U2, st2 = D.unpack_history(D.pack_history(X, U, st))
    assert torch.equal(X2, X) and torch.equal(U2, U) and torch.equal(st2, st)


def _tricky_history(B=5, T=7, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(B, T + 1, 6)) * np.array([1, 1e-5, 1e17, 3, 1e-3, 1.0])
    X[0, 0, 0], X[0, 1, 0], X[1, 2, 1], X[1, 3, 1] = 0.0, -0.0, 1e16, 9999999999999998.0
    X[2, 4, 3], X[2, 5, 3], X[3, 3, 3], X[4, 1, 5] = 0.0001, 0.00001, 123456.0, -2.5e-300
    U = rng.normal(size=(B, T, 2))
    U[0, 0, 0] = 1.0
    return X, U


def test_native_csv_writer_is_byte_identical_to_pandas(tmp_path):
    """traj_dataset_write_csv (multi-threaded, host) writes the same bytes as frames() + DataFrame.to_csv:
    Python-repr floats (fixed / exponent forms, signed zero, 1e16 boundary), empty NaN fields, global ids."""
    X, U = _tricky_history()
    ids = np.arange(40, 45)
    D.write_csv(str(tmp_path / "nat"), X, U, ids, 0.05, native=True, nthreads=3)
    D.write_csv(str(tmp_path / "pd"), X, U, ids, 0.05, native=False)
    for s in ("clean", "noisy"):
        assert (tmp_path / f"nat_{s}.csv").read_bytes() == (tmp_path / f"pd_{s}.csv").read_bytes(), s


def test_native_loader_matches_pandas_loader(tmp_path):
    """load_vehicle_dataset(native=True): the library's parser + numpy grouping gives the pandas path's
    tensors bit for bit (data_loader.py:5-109 semantics), here on shuffled row order and extra rows."""
    import pandas as pd
    rng = np.random.default_rng(1)
    B, T = 12, 30
    X = np.cumsum(rng.normal(size=(B, T + 1, 6)) * 0.01, axis=1)
    U = rng.normal(size=(B, T, 2)) * 0.1
    p = str(tmp_path / "ds")
    D.write_csv(p, X, U, np.arange(B), 0.05)
    for s in ("clean", "noisy"):                       # rows out of order: the loader groups by id
        df = pd.read_csv(f"{p}_{s}.csv")
        df.sample(frac=1.0, random_state=3).sort_values("trajectory_id", kind="stable").to_csv(f"{p}_{s}.csv", index=False)
    a = D.load_vehicle_dataset(f"{p}_noisy.csv", f"{p}_clean.csv", T_steps=25, native=True)
    b = D.load_vehicle_dataset(f"{p}_noisy.csv", f"{p}_clean.csv", T_steps=25)
    for pa, pb in zip(a, b):
        for ta, tb in zip(pa, pb):
            assert ta.dtype == torch.float32 and torch.equal(ta.isnan(), tb.isnan())   # shuffled: last rows inside
            assert torch.equal(ta.nan_to_num(), tb.nan_to_num())
    assert D.load_vehicle_dataset(f"{p}_noisy.csv", f"{p}_clean.csv", T_steps=40, native=True) is None
    assert D.load_vehicle_dataset(str(tmp_path / "missing.csv"), f"{p}_clean.csv", native=True) is None


def test_native_csv_reader_degenerate_files(tmp_path):
    """traj_dataset_read_csv on an empty file and on a header with or without its newline: zero data rows
    parse as OK, asking for rows that are not there is TRAJ_E_ARG (never a read past the buffer)."""
    import ctypes as C
    from trajectory_generation_amd import _lib
    L = _lib.lib()
    cases = {"empty": b"", "header_no_newline": b"X,Y,phi", "header_only": b"X,Y,phi\n"}
    out = (C.c_double * 3)()
    for name, data in cases.items():
        p = tmp_path / f"{name}.csv"
        p.write_bytes(data)
        nc = C.c_int(0)
        assert L.traj_dataset_csv_rows(str(p).encode(), C.byref(nc)) == 0, name
        assert L.traj_dataset_read_csv(str(p).encode(), 0, 3, None, 2) == _lib.TRAJ_OK, name
        assert L.traj_dataset_read_csv(str(p).encode(), 1, 3, out, 2) == _lib.TRAJ_E_ARG, name
    names, buf = D.read_csv_native(str(tmp_path / "header_only.csv"))
    assert names == ["X", "Y", "phi"] and tuple(buf.shape) == (0, 3)
