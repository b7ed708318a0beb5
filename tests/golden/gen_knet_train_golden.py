"""Generate tests/golden/knet_train.npz (KalmanNet training) from the REFERENCE's own code.

Run in the build container only (reads /root/reference):  python tests/golden/gen_knet_train_golden.py

Imported read-only from /root/reference/KalmanNet: kalman_net.KalmanNetNN, vehicle_model.VehicleModel and
pipeline.py's loss functions (_angular_mse_from_real, loss_x_with_angular, compute_composite_loss; a stub
`wandb` module stands in for the logging import).  The weights are tests/_knet_weights.py's seeded set,
the data the B=4 x T=20 sequences of tests/golden/knet.npz, eval mode (dropout off) so the run is
deterministic.  Recorded:
  * the two loss functions on seeded random tensors;
  * the first TBPTT chunk (K=10, composite loss, alpha 0.8): its loss, and per parameter the gradient's
    L2 norm and its first 8 entries;
  * pipeline.py:110-171's chunk losses over T=20 (K=10) with AdamW(lr 1e-4, wd 1e-5) and clipping at 5.0,
    for the 'standard' (step per chunk) and 'accumulation' (one step per trajectory) strategies.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from tests._knet_weights import LIMITS, knet_weights  # noqa: E402

REF = "/root/reference/KalmanNet"


def run_chunks(KN, PL, sysm, g, strategy):
    """pipeline.py:94-171 with the batch, initial posterior and normalization of knet.npz."""
    f32 = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32)   # noqa: E731
    model = KN.KalmanNetNN()
    model.NNBuild(sysm, in_mult_KNet=5, out_mult_KNet=40, hidden_dim_gru=128)
    model.set_normalization(f32(g["x_mean"]), f32(g["x_std"]), f32(g["y_mean"]), f32(g["y_std"]))
    model.load_state_dict({k: torch.tensor(v) for k, v in knet_weights(seed=0).items()})
    model.eval()
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-5)
    x_mean, x_std = f32(g["x_mean"]), f32(g["x_std"])
    y_norm, u = f32(g["y_norm"]), f32(g["u"])
    x_norm = (f32(g["x_true"]) - x_mean) / x_std
    B, T, K = y_norm.shape[0], y_norm.shape[2], 10
    model.batch_size = B
    model.init_hidden_KNet()
    model.InitSequence(f32(g["m1x0"]), T)
    opt.zero_grad()
    outs, xt, yt, losses, grads = [], [], [], [], None
    for t in range(T):
        x_out = model(y_norm[:, :, t].unsqueeze(2), u[:, :, t].unsqueeze(2))
        outs.append(x_out.squeeze(2))
        xt.append(x_norm[:, :, t])
        yt.append(y_norm[:, :, t])
        if (t + 1) % K == 0 or t + 1 == T:
            loss = PL.compute_composite_loss(torch.stack(outs, 2), torch.stack(xt, 2), torch.stack(yt, 2),
                                             x_mean, x_std, 6, 5, 0.8, PL.PHI_IDX)
            if strategy == "accumulation":
                (loss / 2).backward()
            else:
                loss.backward()
            if grads is None:
                grads = {k: p.grad.detach().clone() for k, p in model.named_parameters()}
                if strategy == "accumulation":
                    grads = {k: 2 * v for k, v in grads.items()}
            if strategy != "accumulation":
                torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
                opt.step()
                opt.zero_grad()
            losses.append(float(loss.item()))
            outs, xt, yt = [], [], []
            model.h_Q.detach_()
            model.h_Sigma.detach_()
            model.h_S.detach_()
            model.m1x_posterior.detach_()
    if strategy == "accumulation":
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
        opt.step()
        opt.zero_grad()
    return losses, grads


def main():
    sys.modules["wandb"] = types.ModuleType("wandb")
    sys.path.insert(0, REF)
    import kalman_net as KN
    import pipeline as PL
    import vehicle_model as VM
    torch.set_num_threads(4)
    g = dict(np.load(os.path.join(HERE, "knet.npz")))
    params = dict(VM.Params)
    params.update(LIMITS)
    sysm = VM.VehicleModel(float(g["Ts"]), 20, 20, torch.zeros(6, 1), None, None, None)
    sysm.Params = params

    # loss functions on seeded tensors
    rng = np.random.default_rng(11)
    lx_out = rng.normal(size=(3, 6, 7)).astype(np.float32)
    lx_tgt = rng.normal(size=(3, 6, 7)).astype(np.float32)
    ly_tgt = rng.normal(size=(3, 5, 7)).astype(np.float32)
    lmean = rng.normal(size=(1, 6, 1)).astype(np.float32)
    lstd = (0.5 + rng.random(size=(1, 6, 1))).astype(np.float32)
    lstd[0, 2, 0] = 3.0   # phi spans more than 2 pi: the angular wrap matters
    t = lambda a: torch.tensor(a)   # noqa: E731
    loss_x = float(PL.loss_x_with_angular(t(lx_out), t(lx_tgt), t(lmean), t(lstd), 6))
    loss_c = float(PL.compute_composite_loss(t(lx_out), t(lx_tgt), t(ly_tgt), t(lmean), t(lstd), 6, 5, 0.8))

    losses_std, grads = run_chunks(KN, PL, sysm, g, "standard")
    losses_acc, _ = run_chunks(KN, PL, sysm, g, "accumulation")
    names = sorted(grads)
    np.savez_compressed(
        os.path.join(HERE, "knet_train.npz"),
        loss_in_x_out=lx_out, loss_in_x_tgt=lx_tgt, loss_in_y_tgt=ly_tgt, loss_in_mean=lmean, loss_in_std=lstd,
        loss_x=loss_x, loss_composite=loss_c,
        grad_names=np.array(names), grad_norm=np.array([float(grads[k].norm()) for k in names]),
        grad_head=np.stack([np.pad(grads[k].reshape(-1)[:8].numpy(), (0, max(0, 8 - grads[k].numel())))
                            for k in names]),
        chunk1_loss=losses_std[0], losses_standard=np.array(losses_std), losses_accumulation=np.array(losses_acc))
    print("wrote knet_train.npz", losses_std, losses_acc)


if __name__ == "__main__":
    main()
