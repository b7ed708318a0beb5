"""Trained KalmanNet against the EKF on the config-5 test draw (BASELINE.json configs[4]).

The recipe of KalmanNet/training.py + pipeline.py:287-365 on the build's own data, with the GPU trainer
(knet_train.train_epoch: TBPTT, composite loss alpha 0.8, 'standard' strategy, grad-norm clip 5) and the
fused inference runner:
  * train draw   1024 closed-loop sequences x T (the bench's normalization draw: seed 1, TRAIN_ID_OFFSET ids),
  * val draw     --val sequences (seed 2, ids disjoint from both), validated after every step as
                 validate_epoch does (noisy x(0) init, composite loss), ReduceLROnPlateau(0.5, patience 10,
                 min 1e-7) on it, best weights kept (pipeline.py:357-360),
  * test draw    the bench's 1024 x 200 test sequences (seed 0), hybrid init (test_vehicle.py:123-133):
                 the angular state MSE of the trained network beside the EKF's and the untrained network's.
Architecture: the config-5 network (in_mult 5, out_mult 40, hidden 128 -- test_vehicle.py's NNBuild defaults);
AdamW(lr 1e-4, wd 1e-5), batch 64, --steps optimizer steps (training.py: 500 epochs of one batch each).
Deviation from training.py: sequences of T = 200 (one TBPTT chunk) instead of 1200, to fit one GPU call.

  python tools/knet_train_eval.py [--steps 500] [--out profiles/r03_knet_trained_mse.json]
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trajectory_generation_amd import knet as K  # noqa: E402
from trajectory_generation_amd import knet_eval as KE  # noqa: E402
from trajectory_generation_amd import knet_train as KT  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--val", type=int, default=256)
    ap.add_argument("--out", default="profiles/r03_knet_trained_mse.json")
    ap.add_argument("--save", default="gpurun_out/knet_trained_r03.safetensors")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    Ts, T = 0.01, args.T
    t_gen = time.perf_counter()
    train = KE.make_sequences(1024, T, Ts=Ts, seed=1, id_offset=KE.TRAIN_ID_OFFSET, device=dev)
    val = KE.make_sequences(args.val, T, Ts=Ts, seed=2, id_offset=KE.TRAIN_ID_OFFSET + (1 << 19), device=dev)
    test = KE.make_sequences(1024, 200, Ts=Ts, seed=0, device=dev)
    t_gen = time.perf_counter() - t_gen
    xm, xs, ym, ys, lim = KE.normalization(train)
    norm = {"x_mean": xm, "x_std": xs, "y_mean": ym, "y_std": ys}
    torch.manual_seed(0)
    random.seed(0)
    sysm = K.VehicleModel(Ts, T, T, torch.zeros(6, 1))
    sysm.Params.update(lim)
    model = K.KalmanNetNN(dev)
    model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(xm, xs, ym, ys)

    def evaluate(draw, init):
        """Posteriors (normalized) of the fused runner on a draw; init 'noisy' (validate_epoch) or 'hybrid'."""
        model.eval()
        B = draw["y"].shape[0]
        y_n = ((draw["y"] - ym) / ys).contiguous()
        x_n = (draw["x"] - xm) / xs
        if init == "hybrid":
            m1 = KE.hybrid_init(y_n)
        else:
            x0 = x_n[:, :, 0]
            m1 = (x0 + torch.randn_like(x0) * 0.2).unsqueeze(2)
        out = K.KNetSequenceRunner(model, B).run(y_n, draw["u"].contiguous(), m1, use_graph=False, fused=True)
        return out, x_n, y_n

    def val_loss():
        with torch.no_grad():
            out, x_n, y_n = evaluate(val, "noisy")
            return float(KT.compute_composite_loss(out, x_n, y_n, xm, xs, 6, 5, 0.8))

    out0, x_t, _ = evaluate(test, "hybrid")
    untrained_mse, untrained_db = KE.mse_and_db(out0, x_t, xm, xs)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=10, min_lr=1e-7)
    p = dict(strategy="standard", K_TBPTT=200, T=T, m=6, n=5, CompositionLoss=True, alpha=0.8, N_E=1024,
             N_batch=args.batch, device=dev)
    best, best_state, best_step, hist = float("inf"), None, -1, []
    t_train = 0.0
    for step in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tl, _ = KT.train_epoch(model, opt, train["y"], train["u"], train["x"], norm, p)
        torch.cuda.synchronize()
        t_train += time.perf_counter() - t0
        vl = val_loss()
        sched.step(vl)
        if vl < best:
            best, best_step = vl, step
            best_state = copy.deepcopy(model.state_dict())
        hist.append((step, tl, vl))
        if step % 25 == 0 or step == args.steps - 1:
            print(json.dumps({"step": step, "train": tl, "val": vl, "lr": opt.param_groups[0]["lr"], "best": best}),
                  flush=True)
    model.load_state_dict(best_state)
    out1, x_t, _ = evaluate(test, "hybrid")
    mse, db = KE.mse_and_db(out1, x_t, xm, xs)
    _, ekf_mse, ekf_db = KE.ekf_vs_truth(sysm.Params, Ts, test, xm, xs, ym, ys)
    res = {"what": "KalmanNet trained with the GPU TBPTT trainer (training.py / pipeline.py recipe, T=200) vs the EKF "
                   "on the bench's config-5 test draw (1024 x 200, Ts 0.01)",
           "test": {"trained_mse": mse, "trained_mse_db": db, "ekf_mse": ekf_mse, "ekf_mse_db": ekf_db,
                    "untrained_mse": untrained_mse, "untrained_mse_db": untrained_db},
           "training": {"steps": args.steps, "batch": args.batch, "T": T, "K_TBPTT": 200, "val_sequences": args.val,
                        "best_step": best_step, "best_val_composite": best, "train_s": t_train,
                        "train_seq_steps_per_s": args.steps * args.batch * T / t_train, "data_gen_s": t_gen,
                        "network": "in_mult 5, out_mult 40, hidden 128", "optimizer": "AdamW(1e-4, wd 1e-5)",
                        "scheduler": "ReduceLROnPlateau(0.5, patience 10, min 1e-7) on val"},
           "curve": [{"step": s, "train": a, "val": b} for s, a, b in hist[:: max(1, len(hist) // 40)]]}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    if args.save:
        from safetensors.torch import save_file
        os.makedirs(os.path.dirname(args.save) or ".", exist_ok=True)
        save_file({k: v.detach().contiguous().cpu() for k, v in best_state.items()}, args.save)
    print(json.dumps(res["test"]), flush=True)


if __name__ == "__main__":
    main()
