"""Closed-loop trajectory dataset emitter and its multi-GPU gather (8(e)).

B trajectories per rank run the device-resident closed loop (batch.run_closed_loop: MPC/main.py:85-101
for every trajectory), then the histories are written in the reference's dataset schema
(generation_traj/generation_type1.py:139-158, :295-339):

  clean CSV  t, X, Y, phi, vx, vy, omega, d, delta, trajectory_id
  noisy CSV  t, X, Y, vx, vy, omega, d, delta, trajectory_id        (phi not measured)

one row per time step (T+1 rows per trajectory, the last row's d / delta = NaN), measurement noise
drawn exactly as the reference draws it: ``numpy.random.default_rng(12345 + trajectory_id)``, one
``normal(0, std, T+1)`` vector per channel in the order X, Y, phi, vx, vy, omega (ControlRules,
generation_type1.py:19-33, :312-322).  These files feed merge_datasets.py / data_loader.py unchanged.

Sharding: rank r owns trajectory ids [r B, (r+1) B) (ids and per-trajectory seeds are global, so the
result does not depend on the rank count); the only collective is the final gather of the histories
to rank 0 over RCCL (dist.gather of one fixed-size [B,T+1,9] block per rank; the other ranks receive
nothing), after which rank 0 writes the CSVs.
"""
from __future__ import annotations

import numpy as np

MEAS_NOISE_STD = {"X": 0.05, "Y": 0.05, "phi": 0.003, "vx": 0.010, "vy": 0.003, "omega": 0.030}
NOISE_SEED_BASE = 12345
CLEAN_COLUMNS = ["t", "X", "Y", "phi", "vx", "vy", "omega", "d", "delta", "trajectory_id"]
NOISY_COLUMNS = ["t", "X", "Y", "vx", "vy", "omega", "d", "delta", "trajectory_id"]


def measurement_noise(traj_id: int, n_rows: int, stds=None, seed_base=NOISE_SEED_BASE) -> np.ndarray:
    """[n_rows, 6] noise of one trajectory, generation_type1.py:312-320."""
    s = MEAS_NOISE_STD if stds is None else stds
    rng = np.random.default_rng(seed_base + int(traj_id))
    return np.column_stack([rng.normal(0, s[k], n_rows) for k in ("X", "Y", "phi", "vx", "vy", "omega")])


def frames(X, U, ids, Ts, noise_ids=None):
    """X [B,T+1,6], U [B,T,2] (numpy), ids [B] -> (clean, noisy) pandas DataFrames in the reference
    column order, trajectories stacked in id order.  noise_ids: the ids whose noise draws are added
    (default ids; differs when a filtered dataset is re-indexed)."""
    import pandas as pd
    X = np.asarray(X, dtype=np.float64)
    U = np.asarray(U, dtype=np.float64)
    B, n_rows = X.shape[0], X.shape[1]
    t = np.arange(n_rows) * Ts
    Xn = X + np.stack([measurement_noise(i, n_rows) for i in (ids if noise_ids is None else noise_ids)])
    dU = np.concatenate([U, np.full((B, 1, 2), np.nan)], axis=1)
    tid = np.repeat(np.asarray(ids, dtype=np.int64), n_rows)
    tt = np.tile(t, B)

    def cols(S, with_phi):
        d = {"t": tt, "X": S[:, :, 0].ravel(), "Y": S[:, :, 1].ravel()}
        if with_phi:
            d["phi"] = S[:, :, 2].ravel()
        d.update({"vx": S[:, :, 3].ravel(), "vy": S[:, :, 4].ravel(), "omega": S[:, :, 5].ravel(),
                  "d": dU[:, :, 0].ravel(), "delta": dU[:, :, 1].ravel(), "trajectory_id": tid})
        return pd.DataFrame(d)

    return cols(X, True)[CLEAN_COLUMNS], cols(Xn, False)[NOISY_COLUMNS]


HIST_CHANNELS = 9   # per row: X, Y, phi, vx, vy, omega, d, delta (NaN on the last row), status (-1 on the last row)


def pack_history(X, U, status):
    """X [B,T+1,6], U [B,T,2], status [T,B] -> one [B,T+1,9] float64 block (the unit of the gather)."""
    import torch
    B, T1 = X.shape[0], X.shape[1]
    blk = torch.empty((B, T1, HIST_CHANNELS), dtype=torch.float64, device=X.device)
    blk[:, :, 0:6] = X
    blk[:, :T1 - 1, 6:8] = U
    blk[:, T1 - 1, 6:8] = float("nan")
    blk[:, :T1 - 1, 8] = status.t().to(torch.float64)
    blk[:, T1 - 1, 8] = -1.0
    return blk


def unpack_history(blk):
    """Inverse of pack_history: (X [B,T+1,6], U [B,T,2], status [T,B] int32)."""
    import torch
    return blk[:, :, 0:6], blk[:, :-1, 6:8], blk[:, :-1, 8].t().to(torch.int32)


def gather_to_root(blk, dist=None, dst=0):
    """The dataset's one collective: every rank's fixed-size [B,T+1,9] block goes to
    rank `dst` only (dist.gather -- RCCL over xGMI with the nccl backend, gloo on CPU).  Returns the
    concatenation in rank order (= global trajectory-id order, ids are rank * B + i) on `dst`, None on
    the other ranks; the block itself without a process group.  With a process group the gather runs at
    every world size, 1 included (the same collective path as on 8 GPUs)."""
    if dist is None or not dist.is_initialized():
        return blk
    import torch
    blk = blk.contiguous()
    if dist.get_rank() == dst:
        parts = [torch.empty_like(blk) for _ in range(dist.get_world_size())]
        dist.gather(blk, gather_list=parts, dst=dst)
        return torch.cat(parts, 0)
    dist.gather(blk, dst=dst)
    return None


FAILED_STATUS = 2   # statuses >= 2 (solver error, infeasible, iteration limit, ...): the step kept u_prev


def status_summary(status, ids):
    """status [T,B] (the closed loop's per-step solver status) -> per trajectory (ids [B]): the worst
    status, the number of failed steps (status >= 2) and the first failed step (-1 if none)."""
    st = np.asarray(status)
    T = st.shape[0]
    failed = st >= FAILED_STATUS
    n_failed = failed.sum(axis=0)
    first = np.where(n_failed > 0, np.argmax(failed, axis=0), -1) if T else np.full(st.shape[1], -1)
    worst = st.max(axis=0) if T else np.zeros(st.shape[1], dtype=st.dtype)
    return {"trajectory_id": np.asarray(ids, dtype=np.int64), "worst_status": worst.astype(np.int64),
            "n_failed_steps": n_failed.astype(np.int64), "first_failed_step": first.astype(np.int64)}


def write_status_csv(out_prefix, status, ids, source_ids=None):
    """``{out_prefix}_status.csv`` beside the dataset CSVs (whose reference schema stays unchanged): one row
    per written trajectory -- trajectory_id, source_id (the generation id; differs after filtering),
    worst_status, n_failed_steps, first_failed_step."""
    sm = status_summary(status, source_ids if source_ids is not None else ids)
    with open(f"{out_prefix}_status.csv", "w") as f:
        f.write("trajectory_id,source_id,worst_status,n_failed_steps,first_failed_step\n")
        for i, src, w, n, fs in zip(np.asarray(ids, np.int64), sm["trajectory_id"], sm["worst_status"],
                                    sm["n_failed_steps"], sm["first_failed_step"]):
            f.write(f"{i},{src},{w},{n},{fs}\n")
    return sm


def _closed_loop_gpu(w, T, cfg):
    """This rank's closed loop on the GPU (batch.run_closed_loop, fused launch)."""
    from . import batch as TB
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    return TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, cfg)


def generate(B, T, N=20, Ts=0.05, kind="spline", seed=0, out_prefix=None, dist=None, polish_mode=0,
             closed_loop=None, drop_failed=False, shards=False):
    """Run the closed loop for this rank's B trajectories (ids rank * B .. rank * B + B - 1), gather the
    histories to rank 0 and (rank 0) write ``{out_prefix}_clean.csv`` / ``{out_prefix}_noisy.csv`` and the
    status sidecar ``{out_prefix}_status.csv`` (write_status_csv).

    drop_failed: opt-in (default False, the reference generators' behaviour: generation_type1.py:295-339 writes
      every trajectory, a failed step having kept u_prev as mpc_6stati.py:257-262 returns it; merge_datasets.py
      only offsets the ids of its second file, :41-47, and filters nothing).  True leaves out every trajectory
      with a failed step (status >= 2) and re-indexes the rest 0..n-1 (the contiguous ids data_loader.py reads) --
      each keeps the noise of its generation id, which the sidecar's source_id column records; a warning names
      how many were dropped.  Either way the status sidecar flags the failed trajectories.
    shards: no gather -- every rank writes its own ``{out_prefix}_rank{r}_*.csv`` (global ids; the shards'
      bodies concatenated in rank order are the single file's body) and its sidecar (SURVEY.md 8(e)'s
      per-rank alternative); returns this rank's share on every rank.
    closed_loop(workload, T, cfg) -> dict(X, U, status) runs one rank's share (default: the fused GPU
    closed loop); tests inject a CPU stand-in to exercise the id offsets and the gather.
    Returns (X [W B,T+1,6], U [W B,T,2], status [T,W B]) on rank 0 and None on the other ranks (shards:
    this rank's (X, U, status) everywhere)."""
    from .workload import make_workload
    rank = dist.get_rank() if (dist is not None and dist.is_initialized()) else 0
    w = make_workload(B, N, Ts, kind=kind, seed=seed, id_offset=rank * B)
    cfg = None
    if closed_loop is None:
        from . import batch as TB
        cfg = TB.config_struct(N=N, Ts=Ts, polish_mode=polish_mode)
        closed_loop = _closed_loop_gpu
    if shards and drop_failed:
        raise ValueError("drop_failed re-indexes the whole dataset: it needs the gather (shards=False)")
    res = closed_loop(w, T, cfg)
    if shards:
        X, U, st = res["X"], res["U"], res["status"]
        if out_prefix is not None:
            _write_with_sidecar(f"{out_prefix}_rank{rank}", X, U, st, np.arange(rank * B, rank * B + B), Ts,
                                drop_failed)
        return X, U, st
    blk = gather_to_root(pack_history(res["X"], res["U"], res["status"]), dist)
    if blk is None:
        return None
    X, U, st = unpack_history(blk)
    if out_prefix is not None:
        _write_with_sidecar(out_prefix, X, U, st, np.arange(X.shape[0]), Ts, drop_failed)
    return X, U, st


def _write_with_sidecar(prefix, X, U, st, ids, Ts, drop_failed):
    """CSVs + status sidecar of trajectories `ids` (generation ids); drop_failed re-indexes the kept ones."""
    Xh, Uh = X.cpu().numpy() if hasattr(X, "cpu") else X, U.cpu().numpy() if hasattr(U, "cpu") else U
    sth = st.cpu().numpy() if hasattr(st, "cpu") else np.asarray(st)
    ids = np.asarray(ids, dtype=np.int64)
    if drop_failed:
        keep = np.nonzero((sth >= FAILED_STATUS).sum(axis=0) == 0)[0]
        if keep.size < ids.size:
            import warnings
            warnings.warn(f"{prefix}: drop_failed left out {ids.size - keep.size} of {ids.size} trajectories with a "
                          "failed step and re-indexed the rest (their generation ids: the _status.csv source_id)")
        out_ids = np.arange(keep.size, dtype=np.int64)
        write_csv(prefix, Xh[keep], Uh[keep], out_ids, Ts, noise_ids=ids[keep])
        write_status_csv(prefix, sth[:, keep], out_ids, source_ids=ids[keep])
    else:
        write_csv(prefix, Xh, Uh, ids, Ts)
        write_status_csv(prefix, sth, ids)


def write_csv(out_prefix, X, U, ids, Ts, native=True, nthreads=None, noise_ids=None):
    """``{out_prefix}_clean.csv`` / ``{out_prefix}_noisy.csv`` in the reference schema (see frames).
    native: the library's multi-threaded writer (traj_dataset_write_csv), byte-identical to the pandas
    writer (native=False, frames + DataFrame.to_csv).  noise_ids: see frames."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    U = np.ascontiguousarray(U, dtype=np.float64)
    nids = ids if noise_ids is None else noise_ids
    if not native:
        clean, noisy = frames(X, U, ids, Ts, noise_ids=noise_ids)
        clean.to_csv(f"{out_prefix}_clean.csv", index=False)
        noisy.to_csv(f"{out_prefix}_noisy.csv", index=False)
        return
    import ctypes as C
    import os
    from . import _lib
    B, n_rows = X.shape[0], X.shape[1]
    noise = np.ascontiguousarray(np.stack([measurement_noise(i, n_rows) for i in nids]) if B else
                                 np.zeros((0, n_rows, 6)))
    ids64 = np.ascontiguousarray(ids, dtype=np.int64)
    nt = int(nthreads or min(16, os.cpu_count() or 1))
    p = lambda a: C.c_void_p(a.ctypes.data)   # noqa: E731
    _lib.check(_lib.lib().traj_dataset_write_csv(f"{out_prefix}_clean.csv".encode(), f"{out_prefix}_noisy.csv".encode(),
                                                 B, n_rows - 1, float(Ts), p(X), p(U), p(noise), p(ids64), nt),
               "traj_dataset_write_csv")


def read_csv_native(path, nthreads=None, pin=False):
    """All columns of a dataset CSV as {name: float64 array} through the library's parallel parser
    (traj_dataset_read_csv) into one [rows, C] buffer -- pinned host memory with pin=True."""
    import ctypes as C
    import os
    import torch
    from . import _lib
    with open(path) as f:
        names = f.readline().strip().split(",")
    nc = C.c_int(0)
    rows = int(_lib.lib().traj_dataset_csv_rows(str(path).encode(), C.byref(nc)))
    if rows < 0 or nc.value != len(names):
        raise ValueError(f"{path}: not a dataset CSV ({rows}, {nc.value} columns)")
    buf = torch.empty((rows, len(names)), dtype=torch.float64, pin_memory=pin)
    nt = int(nthreads or min(16, os.cpu_count() or 1))
    _lib.check(_lib.lib().traj_dataset_read_csv(str(path).encode(), rows, len(names), C.c_void_p(buf.data_ptr()), nt),
               "traj_dataset_read_csv")
    return names, buf


def load_vehicle_dataset(noisy_csv_path, clean_csv_path, T_steps=600, train_split=0.7, val_split=0.15, seed=42,
                         device=None, native=False):
    """KalmanNet/data_loader.py:5-109 (load_vehicle_dataset), vectorized: the first T_steps rows of every
    trajectory (ids 0..n-1), y = noisy [X, Y, vx, vy, omega], u = [d, delta], x = clean
    [X, Y, phi, vx, vy, omega] as float32 [n, C, T]; trajectories shuffled by default_rng(seed) and split
    70 / 15 / 15.  Returns ((y, u, x) train, val, test) torch tensors (on ``device`` if given), or None
    when a file or a trajectory is missing, as the reference does."""
    import pandas as pd
    import torch
    if native:
        return _load_native(noisy_csv_path, clean_csv_path, T_steps, train_split, val_split, seed, device)
    try:
        dn = pd.read_csv(noisy_csv_path)
        dc = pd.read_csv(clean_csv_path)
    except FileNotFoundError:
        return None
    n = dn["trajectory_id"].nunique()

    def block(df, cols):
        df = df[df["trajectory_id"] < n]
        df = df.assign(_r=df.groupby("trajectory_id").cumcount())
        df = df[df["_r"] < T_steps]
        counts = df.groupby("trajectory_id").size()
        if len(counts) != n or (counts < T_steps).any():
            raise KeyError("trajectory missing or shorter than T_steps")
        df = df.sort_values(["trajectory_id", "_r"], kind="stable")
        return df[cols].to_numpy(dtype=np.float32).reshape(n, T_steps, len(cols)).transpose(0, 2, 1)

    try:
        y = block(dn, ["X", "Y", "vx", "vy", "omega"])
        u = block(dn, ["d", "delta"])
        x = block(dc, ["X", "Y", "phi", "vx", "vy", "omega"])
    except KeyError:
        return None
    idx = np.arange(n)
    np.random.default_rng(seed).shuffle(idx)
    y, u, x = y[idx], u[idx], x[idx]
    n_tr, n_va = int(n * train_split), int(n * val_split)
    cut = lambda a: (a[:n_tr], a[n_tr:n_tr + n_va], a[n_tr + n_va:])   # noqa: E731
    out = []
    for part in zip(cut(y), cut(u), cut(x)):
        out.append(tuple(torch.tensor(np.ascontiguousarray(p), dtype=torch.float32, device=device) for p in part))
    return tuple(out)


def _load_native(noisy_csv_path, clean_csv_path, T_steps, train_split, val_split, seed, device):
    """load_vehicle_dataset with the library's parser: both files parsed in parallel into pinned host
    buffers, grouped per trajectory with numpy (first T_steps rows of ids 0..n-1, data_loader.py:14-53),
    the three [n, C, T] float32 blocks copied to `device` from pinned memory."""
    import os
    import torch
    if not (os.path.exists(noisy_csv_path) and os.path.exists(clean_csv_path)):
        return None
    pin = device is not None and torch.device(device).type == "cuda"
    blocks = []
    n = None
    for path, cols in ((noisy_csv_path, (["X", "Y", "vx", "vy", "omega"], ["d", "delta"])),
                       (clean_csv_path, (["X", "Y", "phi", "vx", "vy", "omega"],))):
        names, buf = read_csv_native(path, pin=False)
        a = buf.numpy()
        tid = a[:, names.index("trajectory_id")].astype(np.int64)
        if n is None:
            n = int(np.unique(tid).size)
        keep = np.nonzero(tid < n)[0]
        order = keep[np.argsort(tid[keep], kind="stable")]
        counts = np.bincount(tid[keep], minlength=n)
        if counts.size != n or (counts < T_steps).any():
            return None
        first = np.concatenate([[0], np.cumsum(counts)[:-1]])
        rows = order[(first[:, None] + np.arange(T_steps)[None, :]).reshape(-1)]
        for cl in cols:
            idx = [names.index(c) for c in cl]
            blk = a[rows][:, idx].astype(np.float32).reshape(n, T_steps, len(cl)).transpose(0, 2, 1)
            blocks.append(np.ascontiguousarray(blk))
    y, u, x = blocks
    idx = np.arange(n)
    np.random.default_rng(seed).shuffle(idx)
    y, u, x = y[idx], u[idx], x[idx]
    n_tr, n_va = int(n * train_split), int(n * val_split)
    cut = lambda a: (a[:n_tr], a[n_tr:n_tr + n_va], a[n_tr + n_va:])   # noqa: E731

    def dev(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if pin:
            return t.pin_memory().to(device, non_blocking=True)
        return t.to(device) if device is not None else t

    return tuple(tuple(dev(p) for p in part) for part in zip(cut(y), cut(u), cut(x)))
