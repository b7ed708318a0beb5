"""Per-instance timeline of one fused closed-loop launch (diagnostics only): launch span of each
workgroup vs its ADMM iteration total, and how busy the resident slots are."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from trajectory_generation_amd import _lib, batch as TB  # noqa: E402
from trajectory_generation_amd.workload import make_workload  # noqa: E402


def main(B=4096, N=20, Ts=0.05, warm=5, steps=40, kind="spline"):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind=kind)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    x = torch.as_tensor(w["x0"], device=dev).contiguous()
    u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts)
    st = torch.empty((warm + steps, B), dtype=torch.int32, device=dev)
    it = torch.empty((warm + steps, B), dtype=torch.int32, device=dev)
    TB.closed_loop_run(x, u, paths, vref, cfg, None, 0, warm, None, None, st[:warm], it[:warm])
    dbg = torch.zeros((B, 32), dtype=torch.int64, device=dev)
    _lib.lib().traj_debug_set_stamps(C.c_void_p(dbg.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    TB.closed_loop_run(x, u, paths, vref, cfg, None, warm, steps, None, None, st[warm:], it[warm:])
    e1.record()
    torch.cuda.synchronize()
    _lib.lib().traj_debug_set_stamps(None)
    d = dbg.cpu().numpy().astype(float)
    I = it[warm:].cpu().numpy().astype(float)        # [steps, B]
    S = st[warm:].cpu().numpy()
    start = d[:, 22]                                  # by instance
    end = d[:, 23]                                    # by instance
    t0 = start.min()
    ms = e0.elapsed_time(e1)
    print(f"launch {ms:.3f} ms = {ms / steps * 1e3:.1f} us/step; B={B} steps={steps}; status hist {np.bincount(S.reshape(-1), minlength=7).tolist()}")
    tot_it = I.sum(0)
    print("iterations per instance over the launch: median %.0f p90 %.0f p99 %.0f max %.0f (mean %.1f/step)"
          % (np.median(tot_it), np.percentile(tot_it, 90), np.percentile(tot_it, 99), tot_it.max(), tot_it.mean() / steps))
    busy = (end - start) / 100.0                      # us, per instance
    hw = d[:, 24].astype(np.int64)
    xcc = d[:, 25].astype(np.int64) & 0xf
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xf
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    print("busy per instance (us): " + " ".join(f"p{q}={np.percentile(busy, q):.0f}" for q in (1, 10, 50, 90, 99, 100)))
    print("corr(busy, iterations) %.3f" % np.corrcoef(busy, tot_it)[0, 1])
    first = (start - t0) < 2000
    print("first-round instances %d: busy p10 %.0f p50 %.0f p90 %.0f; later: busy p10 %.0f p50 %.0f p90 %.0f"
          % (first.sum(), *np.percentile(busy[first], [10, 50, 90]), *np.percentile(busy[~first], [10, 50, 90])))
    for name, key in (("xcc", xcc), ("se", se), ("simd", simd)):
        vals = sorted(set(key.tolist()))
        print(name, " ".join(f"{v}:{np.median(busy[key == v]):.0f}({(key == v).sum()})" for v in vals))
    # slot sharing: instances that started together on the same SIMD (first round)
    loc = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    fr = np.where(first)[0]
    groups = {}
    for i in fr:
        groups.setdefault(int(loc[i]), []).append(i)
    sizes = np.bincount([len(v) for v in groups.values()])
    print("first-round waves per SIMD:", {k: int(v) for k, v in enumerate(sizes) if v})
    cu_key = (xcc * 8 + se) * 2 * 16 + sh * 16 + cu
    simd_key = cu_key * 4 + simd
    for name, key in (("per CU", cu_key), ("per SIMD", simd_key)):
        groups = {}
        for i in range(B):
            groups.setdefault(int(key[i]), []).append(busy[i])
        means = np.array([np.mean(v) for v in groups.values()])
        spreads = np.array([np.max(v) - np.min(v) for v in groups.values()])
        print(f"{name}: {len(groups)} groups, mean busy p10 {np.percentile(means, 10):.0f} p50 {np.median(means):.0f} "
              f"p90 {np.percentile(means, 90):.0f}; within-group spread p50 {np.median(spreads):.0f} p90 {np.percentile(spreads, 90):.0f}")
    perm = np.arange(B)   # workgroup -> instance is identity unless ordered; end is indexed by instance
    print("workgroup starts (us): " + " ".join(f"p{q}={np.percentile(start - t0, q) / 100:.0f}" for q in (10, 25, 50, 75, 90, 100)))
    print("instance ends   (us): " + " ".join(f"p{q}={np.percentile(end - t0, q) / 100:.0f}" for q in (10, 25, 50, 75, 90, 100)))
    # busy time per instance needs its start: recover via the order kernel's permutation if any
    print("corr(instance end, iterations) %.3f" % np.corrcoef(end, tot_it)[0, 1])
    slots = 2048
    print("ideal (total work / %d slots, work ~ span of the fastest packing): span %.0f us" % (slots, (end.max() - t0) / 100))


if __name__ == "__main__":
    main()
