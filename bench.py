"""bench.py -- MPC steps/sec on B parallel spline-tracking trajectories (BASELINE.json configs[1]).

One bench step = one closed-loop step of MPC/main.py:85-101 for all B trajectories of this rank
(reference window -> linearization -> mpc_step -> Euler plant).  Default: the K timed steps run as ONE
fused traj_closed_loop_run launch (resident workgroups take (step, trajectory) items from a queue;
rollout, Jacobians, condensing, ADMM + polish and the plant update of an item inside one workgroup),
bit-identical to K traj_closed_loop_step calls; --per-step times those calls instead (four launches
per step: rollout_kernel, jac_kernel, order_kernel, solve_kernel).  Inputs and state are resident in
HBM for the whole timed region.  The roofline object is solve_kernel's (the dominant / only kernel),
timed with HIP events the library records on the launch stream.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 4096] [--horizon 20] [--dt 0.05]
  N > 1: python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... --gpus N,
         or plain `python bench.py --gpus N`, which starts the N worker processes itself (RCCL)

Multi-GPU: trajectories are independent, so each rank owns its own B trajectories (ids
rank*B .. rank*B+B-1, weak scaling) with no data-path collective; the ranks only meet at the
timing barriers and the max-over-ranks reduction of the elapsed time.

Prints ONE JSON line (rank 0) with the metric, the roofline of the dominant kernel and the CPU
baseline (the C oracle -- a restatement of the reference path -- on a bounded sample, host cores).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from trajectory_generation_amd import _lib  # noqa: E402
from trajectory_generation_amd import batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
F64_VECTOR_PEAK_TF = 78.6   # MI355X FP64 vector spec (AMD product sheet; the guide lists no f64 figure)
SIMDS, CLOCK_HZ = 1024, 2.4e9   # 256 CUs x 4 SIMDs, max clock (MI355X_MICROARCH.md chip table)


def algorithmic_bytes_per_traj(N: int, kmax: int) -> int:
    """Bytes one trajectory's closed-loop step must move (DESIGN.md 'Roofline'):
    reads  x 6, u_prev 2, vref N+1, path: kind (4 B) + pc 4 + nk (4 B) + knots kmax + coef 4(kmax-1)
    writes x 6, u_prev 2, hist_x 6, hist_u 2, status (4 B), iters (4 B)."""
    doubles = 6 + 2 + (N + 1) + 4 + kmax + 4 * (kmax - 1) + 6 + 2 + 6 + 2
    return 8 * doubles + 4 * 4


def _capacity(n: int) -> int:
    """solve_kernel instance the library launches for 2N QP variables (trajmpc.hip launch_mpc)."""
    return next(c for c in (16, 32, 40, 80) if n <= c)


def _solve_kernel_name(N: int, fused: bool) -> str:
    """The closed loop's solve kernel for horizon N (include/trajmpc.h tiers): the one-wave register-resident
    solve_kernel up to N = 20, the row-split solve_split_kernel<H> for 21 <= N <= 64 (mpc_split.h)."""
    n = 2 * N
    if N < _lib.SPLIT_MIN_N:
        return f"solve_kernel<{_capacity(n)},true>"
    H = 40 if n <= 80 else (48 if n <= 96 else 64)
    return f"solve_split_kernel<{H},true{',true' if fused else ''}>"


def cpu_baseline(w, N, Ts, ntraj, nsteps, polish_mode, warm_start):
    """The oracle (oracle/, C restatement of the reference path + OSQP's ADMM) on host cores."""
    import oracle as O  # test infrastructure: used here only for the CPU-baseline leg
    from trajectory_generation_amd.batch import spline_natural
    O.build()
    paths = []
    for k, c, kn in zip(w["kinds"][:ntraj], w["pcs"][:ntraj], w["knots"][:ntraj]):
        if k == 2:
            paths.append(O.Path(2, (0, 0, 0, 0), xk=kn[0], coef=spline_natural(kn[0], kn[1]).reshape(-1)))
        else:
            paths.append(O.Path(int(k), c))
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cfg = O.cfg(N=N, Ts=Ts, polish_mode=polish_mode, warm_start=warm_start)
    t0 = time.perf_counter()
    O.closed_loop_batch(paths, w["x0"][:ntraj], w["u0"][:ntraj], w["vref"], nsteps, cfg, nthreads=threads)
    dt = time.perf_counter() - t0
    return dict(value=ntraj * nsteps / dt, unit="MPC steps/s", cores=threads, kind="port",
                sample=f"{ntraj} trajectories x {nsteps} closed-loop steps (N={N}, dt={Ts}), "
                       f"C oracle (OpenMP, {threads} threads) = restated mpc_6stati.py + OSQP ADMM/polish, "
                       f"{dt:.2f} s")


def _config1_cases():
    """BASELINE.json configs[0] and MPC/main.py's own loop, as (name, N, Ts, x0, u0, vref, path).
    path: (kind, pcs, knots) of the trajectory's reference (PathSet / oracle kinds)."""
    from trajectory_generation_amd.workload import make_workload as mk
    w = mk(1, 20, 0.05, kind="spline", seed=0, id_offset=0)
    main_x0 = np.array([0.0, 0.5, 0.0, 1.0, 0.0, 0.0])                       # MPC/main.py:80
    main_u0 = np.array([TB.d_steady_state(1.0), 0.0])                          # MPC/main.py:21-22
    return [
        ("configs[0]: one spline trajectory, N=20, dt=0.05", 20, 0.05, w["x0"][0], w["u0"][0], w["vref"],
         (int(w["kinds"][0]), np.asarray(w["pcs"][0], np.float64), w["knots"][0])),
        ("MPC/main.py:72-101: parabola y = 0.1 x^2, N=40, Ts=0.02, ramp vref", 40, 0.02, main_x0, main_u0,
         TB.vref_ramp(40, 0.02), (0, np.array([0.0, 0.0, 0.1, 0.0]), None)),
    ]


def _host_window(path, x_start, N, Ts, vref):
    """MPC/main.py:51-68 on the host for one trajectory: the window the drop-in caller hands mpc_step."""
    from trajectory_generation_amd.workload import spline_eval
    kind, pc, kn = path
    xs = np.zeros(N + 1)
    xs[0] = x_start
    for k in range(N):
        xs[k + 1] = xs[k] + vref[k] * Ts
    if kind == 0:
        ys = pc[0] + xs * (pc[1] + xs * (pc[2] + xs * pc[3]))
        dy = pc[1] + xs * (2.0 * pc[2] + xs * 3.0 * pc[3])
    else:
        coef = TB.spline_natural(kn[0], kn[1])
        yd = [spline_eval(np.asarray(kn[0], np.float64), coef, x) for x in xs]
        ys, dy = np.array([a for a, _ in yd]), np.array([b for _, b in yd])
    return np.stack([xs, ys, np.arctan(dy)], axis=1)


def config1_measure(dev, T=600, cpu=True):
    """BASELINE.json configs[0] (one trajectory, the reference plumbing) on the GPU, three ways:
      dropin  MPC/main.py's loop unchanged after the import swap -- per step the host window, the drop-in
              mpc_step (one QP per call: host -> device copies, the launches, a synchronizing copy back) and
              the drop-in f_cont for the Euler plant; per-call latency of mpc_step and loop steps/s;
      fused   run_closed_loop at B = 1: the T steps in one launch (warm start as the headline, and cold);
      cpu     the C oracle's closed loop on ONE thread, same T steps."""
    from trajectory_generation_amd import mpc_6stati as M
    out = []
    for name, N, Ts, x0, u0, vref, path in _config1_cases():
        rec = {"case": name, "steps": T}
        # --- drop-in loop (MPC/main.py:85-101 with the drop-in module's mpc_step / f_cont)
        for _ in range(3):   # warm the launch path (code objects, allocator)
            M.mpc_step(x0, u0, _host_window(path, x0[0], N, Ts, vref), Ts=Ts, N=N, vref=vref)
        x, u_prev = np.array(x0, np.float64), np.array(u0, np.float64)
        lat, stats = [], []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(T):
            pr = _host_window(path, x[0], N, Ts, vref)
            c0 = time.perf_counter()
            u_cmd, status, _ = M.mpc_step(x, u_prev, pr, Ts=Ts, N=N, params=M.Params, vref=vref)
            lat.append(time.perf_counter() - c0)
            stats.append(status)
            x = x + Ts * M.f_cont(x, u_cmd, M.Params)
            u_prev = u_cmd
        dt = time.perf_counter() - t0
        lat = np.array(lat) * 1e6
        rec["dropin"] = {"steps_per_s": T / dt, "mpc_step_us_median": float(np.median(lat)),
                         "mpc_step_us_p99": float(np.percentile(lat, 99)),
                         "loop_us_per_step": 1e6 * dt / T,
                         "optimal_frac": float(np.mean([s == "optimal" for s in stats])), "final_x": x.tolist()}
        # --- the same closed loop in one fused launch (B = 1)
        kind, pc, kn = path
        paths = TB.PathSet.build([kind], [pc], [kn], device=dev)
        for ws_, key in ((1, "fused"), (0, "fused_cold")):
            cfg = TB.config_struct(N=N, Ts=Ts, warm_start=ws_)
            TB.run_closed_loop(x0, u0, paths, vref, T, cfg)            # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = TB.run_closed_loop(x0, u0, paths, vref, T, cfg)
            torch.cuda.synchronize()
            dtf = time.perf_counter() - t0
            rec[key] = {"steps_per_s": T / dtf, "us_per_step": 1e6 * dtf / T,
                        "iters_mean": float(res["iters"].float().mean()),
                        "final_x": res["X"][0, -1].cpu().numpy().tolist()}
        if cpu:
            rec["cpu_baseline"] = cpu_baseline_config1(N, Ts, x0, u0, vref, path, T)
        out.append(rec)
    return {"what": "BASELINE.json configs[0] / MPC/main.py on one trajectory: the drop-in per-call path, the "
                    "fused closed loop at B=1, and the C oracle on 1 thread", "cases": out}


def cpu_baseline_config1(N, Ts, x0, u0, vref, path, T):
    """The oracle's closed loop (oracle/, C restatement of the reference path) for one trajectory, 1 thread."""
    import oracle as O  # test infrastructure: used here only for the CPU-baseline leg
    O.build()
    kind, pc, kn = path
    p = (O.Path(2, (0, 0, 0, 0), xk=kn[0], coef=TB.spline_natural(kn[0], kn[1]).reshape(-1)) if kind == 2
         else O.Path(int(kind), pc))
    cfg = O.cfg(N=N, Ts=Ts)
    t0 = time.perf_counter()
    r = O.closed_loop(p, x0, u0, vref, T, cfg)
    dt = time.perf_counter() - t0
    return {"steps_per_s": T / dt, "us_per_step": 1e6 * dt / T, "cores": 1, "kind": "port",
            "iters_mean": float(np.mean(r["iters"])), "final_x": r["X"][-1].tolist()}


# KalmanNet (BASELINE.json configs[4]): 1024 sequences x 200 steps, Ts = 0.01, float32
KNET_FLOP_PER_SEQ_STEP = 2 * 3_178_373     # MACs of one gain-network step x 2
FP32_MFMA_PEAK_TFS = 157.3                 # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)
BF16_MFMA_PEAK_TFS = 2500.0                # MI355X dense bf16 matrix peak (the same guide; 2:1-sparse figures excluded)
FC2_TERM_PRODUCTS = 6                      # three-term bf16 form: bf16 MFMA products per f32 product
# fixed clamp limits for the tools' synthetic-input KalmanNet runs (the bench derives its own from data)
KNET_LIMITS = {"x_min": -5.0, "x_max": 40.0, "y_min": -6.0, "y_max": 6.0, "phi_min": -3.2, "phi_max": 3.2,
               "vx_min": 0.0, "vx_max": 3.0, "vy_min": -1.0, "vy_max": 1.0, "omega_min": -6.0, "omega_max": 6.0}


def knet_fc2_flop(B, model):
    """Algorithmic FLOP of one knet_fc2_kernel launch: FC2 = Linear(2H, dH) -> ReLU -> Linear(dH, n m)."""
    H, dH, nm = model.d_hidden_Q, model.d_hidden_FC2, model.n * model.m
    return 2 * B * (2 * H * dH + dH * nm)


def knet_measure(dev, B=1024, T=200, cpu=True, cpu_T=50,
                 traffic_json=os.path.join(HERE, "profiles", "traffic_knet_r05.json"), weights=None,
                 trained_json=os.path.join(HERE, "profiles", "r03_knet_trained_mse.json")):
    """Sequences/s of KalmanNet inference (BASELINE.json configs[4]) on 1024 noisy closed-loop
    trajectories x 200 steps at Ts = 0.01 generated on the GPU (knet_eval.make_sequences: the dataset
    emitter's closed loop + the reference's measurement noise), normalization and clamp limits from a
    separate train draw, seeded-init weights of the reference architecture, all T fused steps replayed
    as one HIP graph.  The same run's posteriors give KalmanNet's MSE (test_vehicle.py:143-158), set
    beside the EKF baseline's on the same measurements.  The roofline object is the dominant kernel's (the FC2
    launch: by default knet_fc2y_kernel, f32 operands as three bf16 terms on the bf16 matrix cores), timed with
    events over standalone launches on the same data; its peak is the bf16 MFMA peak over the six term products
    one f32 product takes, with the f32 MFMA peak beside it."""
    from trajectory_generation_amd import knet as K
    from trajectory_generation_amd import knet_eval as KE
    Ts = 0.01
    train = KE.make_sequences(B, T, Ts=Ts, seed=1, id_offset=KE.TRAIN_ID_OFFSET, device=dev)
    test = KE.make_sequences(B, T, Ts=Ts, seed=0, device=dev)
    xm, xs, ym, ys, lim = KE.normalization(train)
    torch.manual_seed(0)
    sysm = K.VehicleModel(Ts, T, T, torch.zeros(6, 1))
    sysm.Params.update(lim)
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(xm, xs, ym, ys)
    if weights:   # trained weights (tools/knet_train_eval.py --save): the MSE then compares a trained filter
        from safetensors.torch import load_file
        model.load_state_dict({k: v.to(dev) for k, v in load_file(weights).items()})
    model.eval()
    y = ((test["y"] - ym) / ys).contiguous()
    u = test["u"].contiguous()
    m1x0 = KE.hybrid_init(y)
    x_tgt = (test["x"] - xm) / xs
    run = K.KNetSequenceRunner(model, B)
    post = {}

    def timed(**kw):
        run.run(y, u, m1x0, **kw)        # capture + warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        post[kw.get("fused")] = run.run(y, u, m1x0, **kw)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    dt = timed(fused=True)               # the throughput path: 3 launches per step, T steps in one graph
    # the dominant kernel alone (same weights, x2 and workspace as the run): HIP events on the stream
    S, L = run.fs, _lib.lib()
    reps = 50
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fc2 = lambda: _lib.check(L.traj_knet_fc2_f32(ctypes.byref(S["net"]), B, ctypes.c_void_p(S["x2"].data_ptr()),  # noqa
                                                 ctypes.c_void_p(S["ws"][0].data_ptr()), S["ws"][0].numel() * 4,
                                                 ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                             "traj_knet_fc2_f32")
    fc2()
    e0.record()
    for _ in range(reps):
        fc2()
    e1.record()
    torch.cuda.synchronize()
    fc2_ms = e0.elapsed_time(e1) / reps
    fc2_flop = knet_fc2_flop(B, model)
    fc2_tfs = fc2_flop / (fc2_ms * 1e-3) / 1e12
    fc2_mode = L.traj_knet_set_fc2_mode(0)   # (query: set and restore)
    L.traj_knet_set_fc2_mode(fc2_mode)
    if fc2_mode == 0:
        fc2_kernel, fc2_peak = "knet_fc2_kernel<5>", FP32_MFMA_PEAK_TFS
        fc2_peak_note = "f32 MFMA (v_mfma_f32_16x16x4_f32) dense peak"
    else:
        fc2_kernel = "knet_fc2y_kernel<5>" if fc2_mode == 2 else "knet_fc2x_kernel<5>"
        fc2_peak = BF16_MFMA_PEAK_TFS / FC2_TERM_PRODUCTS
        fc2_peak_note = ("f32 FLOP/s ceiling of the three-term form: the dense bf16 MFMA peak / 6 bf16 products per "
                         "f32 product (f32-accurate sums; DESIGN.md 6d)")
    traffic = None
    if os.path.exists(traffic_json):
        try:
            with open(traffic_json) as f:
                tj = json.load(f)
            if tj.get("batch") == B:
                hb = tj.get("hbm_bytes_per_launch", {})
                traffic = hb.get("knet_fc2", hb.get("knet_fc2_kernel"))
        except (OSError, ValueError):
            traffic = None
    dt_step_graph = timed(fused=False)   # module-level step (per-layer launches), one-step graph
    achieved = KNET_FLOP_PER_SEQ_STEP * B * T / dt / 1e12
    knet_mse, knet_db = KE.mse_and_db(post[True], x_tgt, xm, xs)
    mod_mse, _ = KE.mse_and_db(post[False], x_tgt, xm, xs)
    _, ekf_mse, ekf_db = KE.ekf_vs_truth(sysm.Params, Ts, test, xm, xs, ym, ys)
    out = {"metric": f"KalmanNet seq/s (B={B}, T={T})", "value": B / dt, "unit": "sequences/s",
           "ms_per_step": 1e3 * dt / T, "dtype": "f32", "path": "fused (KNetSequenceRunner.run(fused=True))",
           "module_step_graph_value": B / dt_step_graph,
           "config": {"workload": "KalmanNetNN inference (in_mult 5, out_mult 40, hidden 128), seeded-init weights, "
                                  "noisy closed-loop MPC trajectories (knet_eval.make_sequences)", "batch": B, "T": T,
                      "Ts": Ts},
           "mse": knet_mse, "mse_db": knet_db, "mse_module_path": mod_mse, "ekf_mse": ekf_mse, "ekf_mse_db": ekf_db,
           "mse_note": "test_vehicle.py:15-40/149-158 loss on the same 1024 x 200 measurements; KalmanNet weights "
                       + (f"from {os.path.basename(weights)}" if weights else
                          "are the seeded init (no trained weights ship; see 'mse_trained')")
                       + ", the EKF is the build's baseline (f2)",
           "roofline": {"bound": "mfma", "achieved": fc2_tfs, "peak": fc2_peak, "unit": "TFLOP/s",
                        "frac": fc2_tfs / fc2_peak, "traffic": traffic,
                        "kernel": fc2_kernel + " (FC2: Linear 256->10240, ReLU, Linear 10240->30)",
                        "fc2_mode": fc2_mode, "peak_note": fc2_peak_note,
                        "f32_mfma_peak": FP32_MFMA_PEAK_TFS, "frac_of_f32_mfma_peak": fc2_tfs / FP32_MFMA_PEAK_TFS,
                        "kernel_ms": fc2_ms, "flop_per_launch": fc2_flop,
                        "traffic_source": os.path.relpath(traffic_json, HERE) if traffic is not None else None,
                        "whole_step": {"achieved": achieved, "frac": achieved / FP32_MFMA_PEAK_TFS,
                                       "flop_per_seq_step": KNET_FLOP_PER_SEQ_STEP}}}
    if os.path.exists(trained_json):
        # the trained network's MSE on this same test draw, recorded by tools/knet_train_eval.py
        try:
            with open(trained_json) as f:
                tr = json.load(f)
            out["mse_trained"] = dict(tr["test"], source=os.path.relpath(trained_json, HERE),
                                      training=tr.get("training", {}).get("steps"))
        except (OSError, ValueError, KeyError):
            pass
    if cpu:
        import oracle.knet_oracle as KO  # test infrastructure: CPU-baseline leg only
        w = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        p = dict(KO.PARAMS)
        p.update(lim)
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        torch.set_num_threads(threads)
        t0 = time.perf_counter()
        KO.run_sequences(w, p, Ts, y[:, :, :cpu_T].cpu().numpy(), u[:, :, :cpu_T].cpu().numpy(),
                         m1x0.cpu().numpy(), *(a.cpu().numpy() for a in (xm, xs, ym, ys)))
        dtc = (time.perf_counter() - t0) * (T / cpu_T)
        out["cpu_baseline"] = {"value": B / dtc, "unit": "sequences/s", "cores": threads, "kind": "port",
                               "sample": f"{B} sequences x {cpu_T} steps (scaled to T={T}), oracle/knet_oracle.py "
                                         f"(torch CPU float32, {threads} threads); on the 8-thread build host it runs "
                                         f"at the speed of the reference's own KalmanNetNN (199 vs 201 seq/s, "
                                         f"tools/knet_cpu_vs_reference.py)"}
    return out


def knet_predict_measure(dev, B=1024, T=1200, cpu=True, cpu_B=32):
    """test_prediction.py's sliding-window evaluation at its own sizes: T = 1200
    steps per trajectory, H = 200, EVAL_STEP = 100, T_START_EVAL = 50 (10 windows per trajectory), on B
    noisy closed-loop trajectories, test_prediction's architecture (in_mult 10) with seeded-init weights.
    Timed end to end (normalization, initial states, the fused filter over all B trajectories, every
    window's rollout and scores) and the rollout launch alone (HIP events).  The CPU leg is the oracle
    (batched torch float32) on cpu_B trajectories; the reference itself runs the filter at batch size 1
    per trajectory (test_prediction.py:52), slower still."""
    from trajectory_generation_amd import knet as K
    from trajectory_generation_amd import knet_eval as KE
    from trajectory_generation_amd import knet_predict as KP
    Ts = 0.01
    train = KE.make_sequences(256, T, Ts=Ts, seed=3, id_offset=KE.TRAIN_ID_OFFSET, device=dev)
    test = KE.make_sequences(B, T, Ts=Ts, seed=2, device=dev)
    xm, xs, ym, ys, lim = KE.normalization(train)
    torch.manual_seed(0)
    sysm = K.VehicleModel(Ts, T, T, torch.zeros(6, 1))
    sysm.Params.update(lim)
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm, in_mult_KNet=10, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(xm, xs, ym, ys)
    model.eval()
    runner = K.KNetSequenceRunner(model, B)
    args = (model, sysm, test["y"], test["u"], test["x"], xm, xs, ym, ys)
    KP.sliding_window_eval(*args, runner=runner)           # graph capture + warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = KP.sliding_window_eval(*args, runner=runner)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        KP.window_scores(sysm, r["x_est"], xm, xs, test["u"], test["x"])
    e1.record()
    torch.cuda.synchronize()
    roll_ms = e0.elapsed_time(e1) / reps
    W = r["n_windows"]
    out = {"metric": f"sliding-window prediction eval windows/s (B={B}, T={T}, H={KP.H_PRED})",
           "value": W / dt, "unit": "windows/s", "seconds": dt, "windows": W, "rollout_kernel_ms": roll_ms,
           "rollout_windows_per_s": W / (roll_ms * 1e-3), "ade_mean": r["ade_mean"], "fde_mean": r["fde_mean"],
           "config": {"workload": "test_prediction.py main() window loop: KalmanNetNN (in_mult 10) seeded-init weights, "
                                  "noisy closed-loop MPC trajectories (knet_eval.make_sequences)", "batch": B, "T": T,
                      "H": KP.H_PRED, "eval_step": KP.EVAL_STEP, "t_start": KP.T_START_EVAL, "Ts": Ts},
           "note": "ADE / FDE of an untrained filter (plumbing, not quality)"}
    if cpu:
        import oracle.knet_oracle as KO  # test infrastructure: CPU-baseline leg only
        w = {k: v.detach().cpu() for k, v in model.state_dict().items()}
        p = dict(KO.PARAMS)
        p.update(lim)
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        torch.set_num_threads(threads)
        y_n = ((test["y"][:cpu_B] - ym) / ys).cpu().numpy()
        uc, xc = test["u"][:cpu_B].cpu().numpy(), test["x"][:cpu_B].cpu().numpy()
        x0n = r["x0n"][:cpu_B].cpu().numpy()
        t0 = time.perf_counter()
        xe = KO.run_sequences(w, p, Ts, y_n, uc, x0n, *(a.cpu().numpy() for a in (xm, xs, ym, ys)))
        KO.sliding_window_scores(xe, xm.cpu().numpy(), xs.cpu().numpy(), uc, xc, p, Ts, KP.H_PRED, KP.EVAL_STEP,
                                 KP.T_START_EVAL)
        dtc = time.perf_counter() - t0
        wc = cpu_B * (W // B)
        out["cpu_baseline"] = {"value": wc / dtc, "unit": "windows/s", "cores": threads, "kind": "port",
                               "sample": f"{cpu_B} trajectories x {T} steps ({wc} windows), oracle/knet_oracle.py "
                                         f"run_sequences + sliding_window_scores (torch CPU float32, {threads} threads)"}
    return out


def _spawn_workers(n, poll_s=0.2, grace_s=10.0, cmd=None):
    """bench.py --gpus N without a launcher: N worker processes (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous
    on 127.0.0.1), each runs this script on its own GPU over RCCL; the parent never touches the GPU.  It polls
    every worker: on the first non-zero exit the others are terminated (then killed after grace_s) -- a rank
    that dies before or inside the rendezvous must not leave its siblings blocked -- and the parent exits with
    that status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd or ([sys.executable, os.path.abspath(__file__)] + sys.argv[1:]), env=env))
    failed = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c is not None and c != 0]
        if bad:
            failed = bad[0]
            break
        if all(c is not None for c in codes):
            break
        time.sleep(poll_s)
    if failed:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.0, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        sys.exit(failed)


class GpuOps:
    """The bench's device side on this rank's GPU: the closed loop through libtrajmpc.so (fused launches, or
    one traj_closed_loop_step sequence per step), timed with HIP events on the launch stream."""

    def __init__(self, local: int):
        self.dev = TB.require_gpu(f"cuda:{local}")
        torch.cuda.set_device(self.dev)
        if os.environ.get("TRAJ_FUSED_WAVES"):   # experiments: force the fused kernel instance (traj_debug_fused_waves)
            _lib.check(_lib.lib().traj_debug_fused_waves(int(os.environ["TRAJ_FUSED_WAVES"])), "traj_debug_fused_waves")
        if os.environ.get("TRAJ_QUEUE_LEAD"):    # experiments: "steps,per_mille" of the fused queue's lead set
            ls, lp = (int(v) for v in os.environ["TRAJ_QUEUE_LEAD"].split(","))
            _lib.check(_lib.lib().traj_debug_queue_lead(ls, lp), "traj_debug_queue_lead")
        if os.environ.get("TRAJ_RUN_AHEAD"):     # experiments: the fused run's run-ahead levels (traj_debug_run_ahead)
            _lib.check(_lib.lib().traj_debug_run_ahead(int(os.environ["TRAJ_RUN_AHEAD"])), "traj_debug_run_ahead")

    def sync(self):
        torch.cuda.synchronize()

    def setup(self, w, B, N, Ts, T, polish_mode, warm_start=1):
        paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=self.dev)
        st = dict(paths=paths, cfg=TB.config_struct(N=N, Ts=Ts, polish_mode=polish_mode, warm_start=warm_start),
                  x=torch.as_tensor(w["x0"], device=self.dev).contiguous(),
                  u=torch.as_tensor(w["u0"], device=self.dev).contiguous(),
                  vref=torch.as_tensor(np.tile(w["vref"], (B, 1)), device=self.dev).contiguous(),
                  hx=torch.empty((B, T + 1, 6), dtype=torch.float64, device=self.dev),
                  hu=torch.empty((B, T, 2), dtype=torch.float64, device=self.dev),
                  st=torch.empty((T, B), dtype=torch.int32, device=self.dev),
                  it=torch.empty((T, B), dtype=torch.int32, device=self.dev), kmax=int(paths.xk.shape[1]))
        st["hx"][:, 0] = st["x"]
        return st

    def run(self, s, t0, steps, fused):
        """Steps t0 .. t0+steps-1 (one fused launch, or the per-step launches)."""
        if fused:
            TB.closed_loop_run(s["x"], s["u"], s["paths"], s["vref"], s["cfg"], None, t0, steps, s["hx"], s["hu"],
                               s["st"][t0:t0 + steps], s["it"][t0:t0 + steps])
        else:
            for k in range(steps):
                t = t0 + k
                TB.closed_loop_step(s["x"], s["u"], s["paths"], s["vref"], s["cfg"], None, t, s["hx"], s["hu"],
                                    s["st"][t], s["it"][t])

    def kernel_timing(self, steps):
        _lib.check(_lib.lib().traj_debug_kernel_timing(steps), "traj_debug_kernel_timing")

    def kernel_times(self):
        L = _lib.lib()
        kms = (ctypes.c_double * 4)()
        nts = ctypes.c_int(0)
        _lib.check(L.traj_debug_kernel_times(kms, ctypes.byref(nts)), "traj_debug_kernel_times")
        _lib.check(L.traj_debug_kernel_timing(0), "traj_debug_kernel_timing")
        return dict(zip(("rollout_kernel", "jac_kernel", "order_kernel", "solve_kernel"), list(kms)))

    def prepare_dataset(self, w):
        """The dataset leg's reference paths on the device (built before the timed region, as the MPC leg's)."""
        self._ds_paths = (id(w), TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=self.dev))

    def closed_loop(self, w, T, N, Ts, polish_mode):
        """The dataset leg's closed loop of this rank's trajectories: X [B,T+1,6], U [B,T,2], status [T,B]."""
        cached = getattr(self, "_ds_paths", None)
        paths = cached[1] if cached and cached[0] == id(w) else \
            TB.PathSet.build(w["kinds"], w["pcs"], w["knots"], device=self.dev)
        res = TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T,
                                 TB.config_struct(N=N, Ts=Ts, polish_mode=polish_mode))
        return res["X"], res["U"], res["status"]


def dataset_leg(args, w, ops, dist, rank, world):
    """BASELINE.json configs[3] on this node: every rank runs the closed loop of its --batch trajectories
    (ids rank * B + i, the bench workload) for --dataset-steps steps from the initial states, the packed
    [B, T+1, 9] histories go to rank 0 with one dist.gather (RCCL over xGMI), and rank 0 optionally
    writes the CSVs (+ the status sidecar).  With --dataset-csv the per-rank alternative (SURVEY.md 8(e):
    every rank writes its own shard, no gather) is timed beside it.  Generation, gather and CSV writing are
    timed separately (max over ranks)."""
    from trajectory_generation_amd import dataset as D
    B, N, Ts, T = args.batch, args.horizon, args.dt, args.dataset_steps

    def bar():
        ops.sync()
        if dist:
            dist.barrier()
        ops.sync()

    def tmax(v):
        t = torch.tensor([v], dtype=torch.float64, device=ops.dev)
        if dist:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    if hasattr(ops, "prepare_dataset"):
        ops.prepare_dataset(w)
        # torch's copy / cast kernels load their code objects at the first launch (~5 ms here): one tiny untimed
        # pack_history loads them before the timed region (the library preloads its own kernels)
        D.pack_history(torch.zeros((1, 2, 6), dtype=torch.float64, device=ops.dev),
                       torch.zeros((1, 1, 2), dtype=torch.float64, device=ops.dev),
                       torch.zeros((1, 1), dtype=torch.int32, device=ops.dev))
    bar()
    t0 = time.perf_counter()
    X, U, status = ops.closed_loop(w, T, N, Ts, args.polish_mode)
    blk = D.pack_history(X, U, status)
    bar()
    t1 = time.perf_counter()
    full = D.gather_to_root(blk, dist)
    bar()
    t2 = time.perf_counter()
    gen_s, gather_s = tmax(t1 - t0), tmax(t2 - t1)
    csv_s = shard_s = None
    if args.dataset_csv:
        os.makedirs(args.dataset_csv, exist_ok=True)
        if rank == 0:
            Xa, Ua, sta = D.unpack_history(full)
            t3 = time.perf_counter()
            D._write_with_sidecar(os.path.join(args.dataset_csv, "vehicle_mpc"), Xa, Ua, sta, np.arange(Xa.shape[0]),
                                  Ts, False)
            csv_s = time.perf_counter() - t3
        bar()
        t4 = time.perf_counter()
        D._write_with_sidecar(os.path.join(args.dataset_csv, f"vehicle_mpc_rank{rank}"), X, U, status,
                              np.arange(rank * B, rank * B + B), Ts, False)
        shard_s = tmax(time.perf_counter() - t4)
    if rank != 0:
        return None
    Xa, Ua, st = D.unpack_history(full)
    stn = st.cpu().numpy()
    n = world * B * T
    n_failed = int(((stn >= D.FAILED_STATUS).sum(axis=0) > 0).sum())
    return {"what": "configs[3]: closed-loop dataset generation, histories gathered into rank 0",
            "trajectories": world * B, "steps": T, "traj_steps_per_s": n / gen_s, "generate_s": gen_s,
            "gather_s": gather_s, "gather_bytes": int(full.numel() * full.element_size()),
            "csv_s": csv_s, "csv_shards_s": shard_s,
            "csv_note": (f"{n_failed} of {world * B} trajectories have a failed step (status >= 2, u_prev kept as "
                         "mpc_6stati.py:257-262 does); the CSVs hold every trajectory as the reference generators write "
                         "them (dataset.generate's default), the status sidecar flags the failed ones"
                         + ("; csv_s: rank 0 writes the gathered CSVs + status sidecar; csv_shards_s: every rank "
                            "writes its own shard (no gather, failed ones flagged in the sidecar), max over ranks"
                            if args.dataset_csv else "")),
            "status_hist": np.bincount(stn.reshape(-1).astype(np.int64), minlength=7).tolist(),
            "failed_trajectories": n_failed}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4096, help="trajectories per GPU")
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--dt", type=float, default=0.05)
    ap.add_argument("--kind", default="spline", choices=["spline", "mixed", "parabola"])
    ap.add_argument("--polish-mode", type=int, default=0)
    ap.add_argument("--cpu-traj", type=int, default=4096)
    ap.add_argument("--cpu-steps", type=int, default=128)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-knet", action="store_true", help="skip the KalmanNet measurement (configs[4])")
    ap.add_argument("--no-config1", action="store_true",
                    help="skip the one-trajectory measurement (configs[0]: drop-in per call, fused B=1, oracle 1 thread)")
    ap.add_argument("--per-step", action="store_true",
                    help="one traj_closed_loop_step launch sequence per step instead of the fused traj_closed_loop_run")
    ap.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "traffic_r06.json"),
                    help="PMC-measured HBM bytes per launch (from tools/pmc_traffic.py), if present")
    ap.add_argument("--issue-json", default=os.path.join(HERE, "profiles", "sq_f64_r06.json"),
                    help="SQ instruction counts of the fused launch (tools/pmc_f64.sh)")
    ap.add_argument("--stall-json", default=os.path.join(HERE, "profiles", "r06_pmc_stall.json"),
                    help="SQ wave-cycle counters of the fused launch (tools/pmc_stall.sh / pmc_stall.py)")
    ap.add_argument("--knet-traffic-json", default=os.path.join(HERE, "profiles", "traffic_knet_r05.json"),
                    help="PMC-measured HBM bytes of the KalmanNet FC2 launch (tools/pmc_knet_traffic.py)")
    ap.add_argument("--knet-weights", default=None,
                    help="safetensors of trained KalmanNet weights (tools/knet_train_eval.py --save) for configs[4]")
    ap.add_argument("--dataset-steps", type=int, default=240,
                    help="configs[3] leg: closed-loop dataset generation of --batch trajectories per GPU over this "
                         "many steps, then the histories gathered into rank 0 (0 disables)")
    ap.add_argument("--dataset-csv", default=None,
                    help="directory: rank 0 also writes the dataset CSVs there (timed separately)")
    ap.add_argument("--no-cold", action="store_true",
                    help="skip the reference-semantics (cold-start) pass reported as 'cold'")
    ap.add_argument("--no-config3", dest="config3", action="store_false",
                    help="skip the configs[2] object (N = 40, mixed references, same steps / warmup; one GPU)")
    ap.add_argument("--config3-traffic-json", default=os.path.join(HERE, "profiles", "traffic_r06_n40.json"))
    ap.add_argument("--config3-issue-json", default=os.path.join(HERE, "profiles", "sq_f64_r06_n40.json"))
    ap.add_argument("--config3-stall-json", default=os.path.join(HERE, "profiles", "r06_pmc_stall_n40.json"))
    ap.add_argument("--config3-cpu-traj", type=int, default=512)
    ap.add_argument("--config3-cpu-steps", type=int, default=16)
    ap.add_argument("--no-host-io", dest="host_io", action="store_false",
                    help="skip the end-to-end (H2D + run + D2H) variant of the headline ('host_io')")
    ap.add_argument("--dist-timeout", type=float, default=600.0,
                    help="seconds before a process-group rendezvous or collective gives up (N > 1)")
    args = ap.parse_args(argv)
    # the profiles of another horizon (config 3's N = 40: traffic_r06_n40.json, sq_f64_r06_n40.json) when the
    # defaults are in use and such a file exists
    if args.horizon != 20:
        for k in ("traffic_json", "issue_json"):
            v = getattr(args, k)
            alt = v[:-5] + f"_n{args.horizon}.json"
            if v == ap.get_default(k) and os.path.exists(alt):
                setattr(args, k, alt)
    return args


def main(argv=None, ops_factory=None, backend=None):
    """The bench.  ops_factory(local_rank) gives the device side (default GpuOps); backend the process-group
    backend (default nccl = RCCL; tests pass gloo with a CPU stand-in)."""
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start one worker process per GPU before anything in this process touches the GPU
        return _spawn_workers(args.gpus)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env != args.gpus and args.gpus != 1:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries the one JSON line only: what libraries print there while the bench runs (RCCL prints its
    # version banner to stdout when a communicator is created) is routed to stderr until the line is written
    sys.stdout.flush()
    saved_stdout = os.dup(1)
    os.dup2(2, 1)
    try:
        out = _main_ranked(args, ops_factory, backend, world_env, rank, local)
    finally:
        sys.stdout.flush()
        os.dup2(saved_stdout, 1)
        os.close(saved_stdout)
    if out is not None:
        print(json.dumps(out), flush=True)
    return out


def _main_ranked(args, ops_factory, backend, world_env, rank, local):
    """This rank's process group (if any), device side and bench; rank 0 returns the record."""
    dist = None
    world = 1
    backend = backend or os.environ.get("TRAJ_BENCH_BACKEND", "nccl")
    # TRAJ_BENCH_PG=1: a process group even at world size 1 (exercises the RCCL rendezvous, the barriers and the
    # MAX all-reduce on a one-GPU box -- tools/r03_rccl.sh; the driver's N = 1 run does not set it)
    if world_env > 1 or os.environ.get("TRAJ_BENCH_PG") == "1":
        import datetime
        import torch.distributed as dist
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=args.dist_timeout), **kw)
        world = dist.get_world_size()
        assert world == world_env
    ops = (ops_factory or GpuOps)(local)
    try:
        out = bench_run(args, ops, dist, rank, world)
    finally:
        if dist:
            dist.destroy_process_group()
    return out


def _load_profile(path, **want):
    """A profile JSON (tools/pmc_*.py output) if it describes this launch, else None -- and why, so that a line whose
    roofline.traffic / roofline.issue is null says which file was looked at and what did not match."""
    if not path or not os.path.exists(path):
        return None, f"{os.path.relpath(os.path.abspath(path), HERE) if path else path}: not found"
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError) as e:
        return None, f"{os.path.relpath(path, HERE)}: unreadable ({e})"
    for k, v in want.items():
        have = d.get(k, 20 if k == "horizon" else None)
        if k == "fused":
            have = bool(d.get("fused", False))
        if have != v:
            return None, f"{os.path.relpath(path, HERE)}: {k} = {have}, this launch has {v}"
    return d, None


def f64_flop_algorithmic(N, K):
    """F(N, K) = N (60 + 150) + 72 N (N + 1) + (N + 1)(72 N + 24 N^2) + 8 N^3 / 3 + K (8 N^2 + 20 N)
    algorithmic f64 FLOP per MPC step, K = mean ADMM iterations."""
    return N * 210 + 72 * N * (N + 1) + (N + 1) * (72 * N + 24 * N * N) + 8 * N ** 3 / 3 + K * (8 * N * N + 20 * N)


def mpc_leg(args, ops, dist, rank, world, N, kind, traffic_json, issue_json, stall_json=None, with_cold=True):
    """One closed-loop MPC measurement: --warmup untimed steps, then EXACTLY --steps timed steps bracketed by barrier +
    synchronize on both sides (max over ranks), state resident in HBM; the roofline object of the dominant kernel
    (solve_kernel, HIP events on its launch stream), the PMC traffic / issue profiles if they describe this launch,
    and (with_cold) the same command with cold rho.  Returns (record, state, workload, iterations, statuses)."""
    Ts, B = args.dt, args.batch
    w = make_workload(B, N, Ts, kind=kind, seed=0, id_offset=rank * B)
    T = args.warmup + args.steps
    fused = not args.per_step

    def timed_pass(warm_start, timing):
        """W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier + synchronize on both
        sides; the elapsed time is the max over ranks."""
        s = ops.setup(w, B, N, Ts, T, args.polish_mode, warm_start=warm_start)
        if args.warmup:
            ops.run(s, 0, args.warmup, fused)
        ops.sync()
        if dist:
            dist.barrier()
        ops.sync()
        if timing:
            ops.kernel_timing(args.steps)
        t0 = time.perf_counter()
        ops.run(s, args.warmup, args.steps, fused)   # fused: all K steps in one launch (= K step launches)
        ops.sync()
        if dist:
            dist.barrier()
        ops.sync()
        elapsed = time.perf_counter() - t0
        if dist:
            e = torch.tensor([elapsed], dtype=torch.float64, device=ops.dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            elapsed = float(e.item())
        return s, elapsed

    # the headline: the closed loop's warm start (each step's ADMM from the rho the previous step adapted to;
    # the polished optimum does not depend on rho).  The reference solves cold every step -- a new cp.Problem
    # per call makes its warm_start=True a no-op (mpc_6stati.py:252-256) -- reported beside it ("cold").
    s, elapsed = timed_pass(1, True)
    kernels_ms = ops.kernel_times()
    cold = None
    if with_cold:
        s_cold, el_cold = timed_pass(0, False)
        ic = s_cold["it"][args.warmup:].cpu().numpy().reshape(-1)
        cold = {"what": "the same command with warm_start=0 (cold rho every step, the reference's effective "
                        "semantics, mpc_6stati.py:252-256)",
                "value": world * B * args.steps / el_cold, "ms_per_step": 1e3 * el_cold / args.steps,
                "iters_mean": float(ic.mean()), "iters_p99": float(np.percentile(ic, 99)), "iters_max": int(ic.max()),
                "status_hist": np.bincount(s_cold["st"][args.warmup:].cpu().numpy().reshape(-1), minlength=7).tolist()}
    if fused:   # one launch = args.steps closed-loop steps, linearization inside the solve kernel
        kernels_ms = {"solve_kernel": kernels_ms["solve_kernel"]}
    kern_ms = kernels_ms["solve_kernel"]
    steps_per_launch = args.steps if fused else 1
    iters = s["it"][args.warmup:].cpu().numpy().reshape(-1)
    stat = s["st"][args.warmup:].cpu().numpy().reshape(-1)
    value = world * B * args.steps / elapsed
    kmax = s["kmax"]
    bytes_launch = B * algorithmic_bytes_per_traj(N, kmax) * steps_per_launch
    achieved = bytes_launch / (kern_ms * 1e-3) / 1e9 if kern_ms > 0 else None
    traffic = traffic_step = None
    tj, traffic_why = _load_profile(traffic_json, horizon=N, fused=fused)
    if tj is not None:
        if fused and tj.get("hbm_bytes_per_instance_step"):
            # PMC bytes per instance-step of the profiled fused launch x this launch's instance-steps
            traffic = float(tj["hbm_bytes_per_instance_step"]) * B * steps_per_launch
            traffic_step = float(tj["hbm_bytes_per_instance_step"]) * B
        elif tj.get("batch") == B and int(tj.get("steps_per_launch", 1)) == steps_per_launch:
            traffic = tj.get("hbm_bytes_per_kernel", {}).get("solve_kernel")
            traffic_step = tj.get("hbm_bytes_per_launch")
        else:
            traffic_why = f"{os.path.relpath(traffic_json, HERE)}: batch / steps_per_launch differ from this launch"
    issue = None
    ij, issue_why = _load_profile(issue_json, batch=B, horizon=N)
    if ij is not None:
        try:
            # solve_kernel is VALU-issue/latency bound: the issued f64 lane-FLOP rate against the f64
            # vector peak, and the VALU issue slots used (4 cycles per wave64 instruction)
            fl = ij["f64_flop_issued_per_step"] * value / world / 1e12
            K = float(iters.mean())
            f_alg = f64_flop_algorithmic(N, K)
            fa = f_alg * value / world / 1e12
            issue = {"what": "solve_kernel issue side (PMC SQ_INSTS_VALU*, per instance-step x steps/s)",
                     "f64_tflops_issued": fl, "f64_peak_tflops": F64_VECTOR_PEAK_TF,
                     "f64_frac": fl / F64_VECTOR_PEAK_TF,
                     "f64_flop_algorithmic_per_step": f_alg, "f64_tflops_algorithmic": fa,
                     "f64_frac_algorithmic": fa / F64_VECTOR_PEAK_TF,
                     "issued_over_algorithmic": ij["f64_flop_issued_per_step"] / f_alg,
                     "valu_insts_per_step": ij["valu_insts_per_step"],
                     "valu_issue_frac": ij["valu_insts_per_step"] * 4 * value / world / (SIMDS * CLOCK_HZ),
                     "source": os.path.relpath(issue_json, HERE)}
            if "f64_valu_insts_per_step" in ij:
                # SIMD VALU busy time on CDNA4 (MI355X_MICROARCH.md, per-instruction constants): a wave64
                # f64 instruction holds the 16-lane f64 pipe 4 cycles, any other VALU instruction the
                # 32-wide SIMD 2 cycles
                f64i = ij["f64_valu_insts_per_step"]
                issue["simd_valu_busy_frac"] = ((f64i * 4 + (ij["valu_insts_per_step"] - f64i) * 2) * value / world
                                                / (SIMDS * CLOCK_HZ))
        except (KeyError, TypeError, ZeroDivisionError) as e:
            issue, issue_why = None, f"{os.path.relpath(issue_json, HERE)}: missing field ({e})"
    if issue is not None and fused and stall_json:
        sj, stall_why = _load_profile(stall_json)
        if sj is not None and sj.get("batch", B) == B and sj.get("horizon", 20) == N:
            try:
                sc = sj["counters"]
                # measured SIMD VALU occupancy of the profiled launch: SQ_ACTIVE_INST_VALU (quad-cycles, summed over
                # waves) x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs) -- no clock assumption (MI355X_MICROARCH.md)
                issue["simd_valu_active_frac_pmc"] = sc["SQ_ACTIVE_INST_VALU"] * 4.0 / (SIMDS * sc["GRBM_GUI_ACTIVE"] / 8.0)
                issue["wave_cycle_split_pmc"] = {k: sc[k] / sc["SQ_WAVE_CYCLES"] for k in
                                                 ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")}
                issue["stall_source"] = os.path.relpath(stall_json, HERE)
            except (KeyError, ZeroDivisionError):
                pass
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved is not None else None, "traffic": traffic,
            "kernel": _solve_kernel_name(N, fused) + (
                f" (fused closed loop, {steps_per_launch} steps per launch)" if fused else ""),
            "kernel_ms": kern_ms, "steps_per_launch": steps_per_launch,
            "bytes_per_launch": bytes_launch, "kernels_ms": kernels_ms, "traffic_step": traffic_step,
            "traffic_source": os.path.relpath(os.path.abspath(traffic_json), HERE) if traffic is not None else None,
            "issue": issue}
    if traffic is None:
        roof["traffic_rejected"] = traffic_why
    if issue is None:
        roof["issue_rejected"] = issue_why
    rec = {"value": value, "ms_per_step": 1e3 * elapsed / args.steps, "roofline": roof,
           "solver_stats": {"iters_mean": float(iters.mean()), "iters_p99": float(np.percentile(iters, 99)),
                            "iters_max": int(iters.max()), "status_hist": np.bincount(stat, minlength=7).tolist()},
           "cold": cold}
    return rec, s, w


def host_io_measure(args, ops, w, N, reps=3):
    """SURVEY.md 8(d)'s end-to-end variant of the headline (kernel + H2D/D2H inside the timed region): the host hands
    over x0, u_prev, the reference paths and vref in pageable numpy arrays, the W + K closed-loop steps run (the same
    fused launches as the headline), and the histories X [B,T+1,6], U [B,T,2], status / iters [T,B] come back to
    host numpy.  Median of `reps` runs; the headline's `value` keeps the inputs resident in HBM (the task's contract)."""
    B, Ts = args.batch, args.dt
    T = args.warmup + args.steps
    fused = not args.per_step
    times = []
    for _ in range(reps + 1):
        ops.sync()
        t0 = time.perf_counter()
        s = ops.setup(w, B, N, Ts, T, args.polish_mode, warm_start=1)       # H2D: states, paths, vref
        if args.warmup:
            ops.run(s, 0, args.warmup, fused)
        ops.run(s, args.warmup, args.steps, fused)
        out = [s[k].cpu().numpy() for k in ("hx", "hu", "st", "it")]      # D2H: the histories
        times.append(time.perf_counter() - t0)
    dt = float(np.median(times[1:]))
    h2d = sum(int(np.asarray(w[k]).nbytes) for k in ("x0", "u0")) + B * (N + 1) * 8
    d2h = sum(int(a.nbytes) for a in out)
    return {"what": "end to end from host arrays: upload x0 / u_prev / paths / vref, W + K closed-loop steps (fused), "
                    "download X / U / status / iters histories (SURVEY.md 8(d) 'kernel + H2D/D2H inside the timed region')",
            "value": B * T / dt, "unit": "MPC steps/s", "steps": T, "seconds": dt, "d2h_bytes": d2h,
            "h2d_bytes_min": h2d, "reps": reps}


def bench_run(args, ops, dist, rank, world):
    """One rank's bench: warmup, the timed region bracketed by barrier + synchronize on both sides, the
    max-over-ranks elapsed time, the dataset leg; rank 0 returns the JSON record (None elsewhere)."""
    N, Ts, B = args.horizon, args.dt, args.batch
    fused = not args.per_step
    stall = args.stall_json if (N == 20 and B == 4096) else None    # (the profiled config)
    rec, s, w = mpc_leg(args, ops, dist, rank, world, N, args.kind, args.traffic_json, args.issue_json, stall,
                        with_cold=not args.no_cold)
    dataset = dataset_leg(args, w, ops, dist, rank, world) if args.dataset_steps > 0 else None
    # config 3 (BASELINE.json configs[2]): 4096 mixed sinusoid / parabola references, N = 40, same K / W -- its own line
    # object beside the headline, measured by the same timed region (one GPU)
    cfg3 = None
    if args.config3 and world == 1 and not (N == 40 and args.kind == "mixed"):
        r3, _, w3 = mpc_leg(args, ops, dist, rank, world, 40, "mixed", args.config3_traffic_json,
                            args.config3_issue_json, args.config3_stall_json, with_cold=False)
        cfg3 = dict({"metric": f"MPC steps/sec (batch={B}, N=40, mixed sinusoid/parabola references)",
                     "unit": "MPC steps/s", "steps": args.steps, "warmup": args.warmup,
                     "config": {"workload": f"closed-loop mixed (50 % sinusoid, 50 % parabola) tracking MPC, {B} "
                                            f"trajectories, N=40, dt={Ts}s (BASELINE.json configs[2])",
                                "horizon": 40, "dt": Ts, "batch": B}}, **r3)
        if not args.no_cpu:
            cfg3["cpu_baseline"] = cpu_baseline(w3, 40, Ts, min(args.config3_cpu_traj, B), args.config3_cpu_steps,
                                                args.polish_mode, 1)
    host_io = host_io_measure(args, ops, w, N) if (args.host_io and world == 1 and fused) else None
    if rank != 0:
        return None

    out = {
        "metric": "MPC steps/sec (batch=4096, N=20)" if (B == 4096 and N == 20) else f"MPC steps/sec (batch={B}, N={N})",
        "value": rec["value"],
        "unit": "MPC steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": rec["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": f"closed-loop {args.kind}-tracking MPC, {B} trajectories/GPU, N={N}, dt={Ts}s",
                   "global_batch": world * B, "horizon": N, "dt": Ts, "parallelism": f"shard{world}",
                   "solver": f"ADMM(OSQP restated)+polish mode {args.polish_mode}, fp64",
                   "warm_start": "rho carried from the instance's previous step (closed loop); cold: see 'cold'",
                   "launch": "fused traj_closed_loop_run" if fused else "traj_closed_loop_step per step",
                   "timed_region": "device-resident state: x0 / u_prev / paths / vref uploaded and histories left in "
                                   "HBM outside the timed region (H2D / D2H excluded); the end-to-end variant with both "
                                   "inside is 'host_io'"},
        "roofline": rec["roofline"],
        "solver_stats": rec["solver_stats"],
    }
    out["cold"] = rec["cold"]
    out["dataset"] = dataset
    out["host_io"] = host_io
    out["config3"] = cfg3
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(w, N, Ts, min(args.cpu_traj, B), args.cpu_steps, args.polish_mode,
                                           s["cfg"].warm_start)
    else:
        out["cpu_baseline"] = None
    if not args.no_knet and world == 1:
        out["knet"] = knet_measure(ops.dev, cpu=not args.no_cpu, traffic_json=args.knet_traffic_json,
                                   weights=args.knet_weights)
        out["knet"]["prediction"] = knet_predict_measure(ops.dev, cpu=not args.no_cpu)
    if not args.no_config1 and world == 1:
        out["config1"] = config1_measure(ops.dev, cpu=not args.no_cpu)
    return out




if __name__ == "__main__":
    main()
