"""Work-item timeline of one fused closed-loop launch (traj_debug_set_item_stamps; diagnostics only).

  python tools/item_timeline.py [steps] [warmup] [B]

Where the slot time of the launch goes: working on items, waiting for an instance's previous step,
idle after the queue drained; and the chain of the instance that finishes last (per step: drawn,
start, end, ADMM iterations)."""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def decode(q, B, S, L, H):
    """Work item q -> (step, rank): the fused queue order of mpc_solve.h (heavy ranks < H lead by L)."""
    L = min(L, S) if H > 0 else 0
    H = H if L > 0 else 0
    P = L * H
    step = np.empty_like(q)
    rank = np.empty_like(q)
    a = q < P
    step[a], rank[a] = q[a] // max(H, 1), q[a] % max(H, 1)
    q1 = q - P
    full = (S - L) * B
    b = (~a) & (q1 < full)
    lv, r = q1[b] // B, q1[b] % B
    step[b], rank[b] = np.where(r < H, lv + L, lv), r
    c = (~a) & (q1 >= full)
    q2 = q1[c] - full
    step[c], rank[c] = (S - L) + q2 // (B - H), H + q2 % (B - H)
    return step, rank


def main(steps=20, warm=5, B=4096, N=20, Ts=0.05, kind="spline", out=None, lead=(1, 100)):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind=kind)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    st = torch.empty((warm + steps, B), dtype=torch.int32, device=dev)
    it = torch.empty((warm + steps, B), dtype=torch.int32, device=dev)
    if warm:
        TB.closed_loop_run(x, u, paths, vref, cfg, None, 0, warm, None, None, st[:warm], it[:warm])
    items = torch.zeros((steps * B, 4), dtype=torch.int64, device=dev)
    _lib.lib().traj_debug_queue_lead(*lead)
    if os.environ.get("TL_RA"):
        _lib.lib().traj_debug_run_ahead(int(os.environ["TL_RA"]))
    if os.environ.get("TL_WAVES"):
        _lib.lib().traj_debug_fused_waves(int(os.environ["TL_WAVES"]))
    perm_ws = TB.workspace(B, N, dev)
    _lib.lib().traj_debug_set_item_stamps(C.c_void_p(items.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    TB.closed_loop_run(x, u, paths, vref, cfg, None, warm, steps, None, None, st[warm:], it[warm:])
    e1.record()
    torch.cuda.synchronize()
    _lib.lib().traj_debug_set_item_stamps(None)
    ms = e0.elapsed_time(e1)
    d = items.cpu().numpy().astype(np.float64)
    # perm used by the launch: rank -> instance (order_kernel output, in the workspace after the warm record)
    off = (B * N * 66 + B * 4) * 8
    perm = perm_ws.view(torch.uint8)[off:off + 4 * B].view(torch.int32).cpu().numpy() if warm else np.arange(B)
    I = it[warm:].cpu().numpy()                       # [steps, B] by instance
    drawn, start, end, slot = d[:, 0], d[:, 1], d[:, 2], d[:, 3].astype(np.int64)
    t0 = drawn.min()
    drawn, start, end = (drawn - t0) / 100.0, (start - t0) / 100.0, (end - t0) / 100.0   # us
    span = end.max()
    work = end - start
    wait = start - drawn
    nslots = slot.max() + 1
    q = np.arange(steps * B)
    H = (B * lead[1]) // 1000 if warm else 0
    stp, rk = decode(q, B, steps, lead[0], min(H, B - 1))
    inst = perm[rk]
    iters = I[stp, inst]
    res = {"launch_ms_events": ms, "span_us": span, "steps": steps, "B": B, "slots": int(nslots),
           "items": int(steps * B)}
    slot_time = nslots * span
    res["slot_time_split"] = {"working": work.sum() / slot_time, "waiting": wait.sum() / slot_time,
                              "idle_or_between": 1 - (work.sum() + wait.sum()) / slot_time}
    # per slot: time of its last item end (when the slot went idle for good)
    last_end = np.zeros(nslots)
    np.maximum.at(last_end, slot, end)
    res["slot_drain_us"] = {p: float(np.percentile(last_end, p)) for p in (1, 10, 50, 90, 99, 100)}
    res["item_work_us_by_step"] = [float(np.median(work[stp == s])) for s in range(steps)]
    res["item_iters_mean_by_step"] = [float(iters[stp == s].mean()) for s in range(steps)]
    res["wait_us"] = {"mean": float(wait.mean()), "p99": float(np.percentile(wait, 99)), "max": float(wait.max()),
                      "items_waiting_gt_5us": int((wait > 5).sum())}
    # fit item work ~ a + b * iters
    A = np.stack([np.ones_like(iters, dtype=float), iters.astype(float)], 1)
    coef, *_ = np.linalg.lstsq(A, work, rcond=None)
    res["work_fit_us"] = {"per_item": float(coef[0]), "per_iter": float(coef[1])}
    # the chain of the last instance to finish
    endi = np.zeros(B)
    np.maximum.at(endi, inst, end)
    crit = int(np.argmax(endi))
    sel = np.where(inst == crit)[0]
    sel = sel[np.argsort(stp[sel])]
    chain = []
    for j in sel:
        chain.append({"step": int(stp[j]), "rank": int(rk[j]), "drawn": round(drawn[j], 1), "start": round(start[j], 1),
                      "end": round(end[j], 1), "iters": int(iters[j])})
    res["critical_instance"] = {"b": crit, "total_iters": int(I[:, crit].sum()), "chain": chain,
                                "chain_work_us": float(work[sel].sum()), "chain_wait_us": float(wait[sel].sum()),
                                "gaps_us": float(sum(start[sel[i + 1]] - end[sel[i]] for i in range(len(sel) - 1)))}
    # busy slots over time (working), 20 bins
    bins = np.linspace(0, span, 21)
    busy = []
    for lo, hi in zip(bins[:-1], bins[1:]):
        ov = np.clip(np.minimum(end, hi) - np.maximum(start, lo), 0, None).sum()
        busy.append(round(float(ov / ((hi - lo) * nslots)), 3))
    res["busy_frac_by_time_bin"] = busy
    js = json.dumps(res)
    print(js)
    if out:
        with open(out, "w") as f:
            f.write(js)


if __name__ == "__main__":
    a = [int(v) for v in sys.argv[1:4]]
    # TL_N / TL_KIND: horizon and reference kind (config 3: TL_N=40 TL_KIND=mixed)
    main(*a, N=int(os.environ.get("TL_N", 20)), kind=os.environ.get("TL_KIND", "spline"),
         out=os.environ.get("TL_OUT"))
