"""Per-phase cycle breakdown of the fused MPC kernel (uses traj_debug_set_stamps; diagnostics only)."""
import sys, os, ctypes as C
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from trajectory_generation_amd import batch as TB, _lib
from trajectory_generation_amd.workload import make_workload

def main(B=int(os.environ.get("PP_B", 4096)), N=20, Ts=0.05, warm=5, kind="spline", polish_mode=0, fused=0):
    dev = TB.require_gpu()
    w = make_workload(B, N, Ts, kind=kind)
    paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
    x = torch.as_tensor(w["x0"], device=dev).contiguous(); u = torch.as_tensor(w["u0"], device=dev).contiguous()
    vref = torch.as_tensor(np.tile(w["vref"], (B, 1)), device=dev).contiguous()
    cfg = TB.config_struct(N=N, Ts=Ts, polish_mode=polish_mode)
    for t in range(warm):
        TB.closed_loop_step(x, u, paths, vref, cfg, None, t)
    dbg = torch.zeros((B, 32), dtype=torch.int64, device=dev)
    _lib.lib().traj_debug_set_stamps(C.c_void_p(dbg.data_ptr()))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    if fused:   # one fused launch of `fused` steps; the stamps hold each instance's last step
        TB.closed_loop_run(x, u, paths, vref, cfg, None, warm, fused)
    else:
        TB.closed_loop_step(x, u, paths, vref, cfg, None, warm)
    e1.record()
    torch.cuda.synchronize()
    _lib.lib().traj_debug_set_stamps(None)
    d = dbg.cpu().numpy()
    names = ["inputs", "condense", "scale", "solve", "outputs"]
    idx = [0, 1, 4, 5, 6, 7]
    ph_all = np.diff(d[:, idx], axis=1)
    # an item that ends before the ADMM (solver error on non-finite data, infeasible up front) writes no solve stamps:
    # its slots hold an earlier item's values (non-monotone phases, maxima of 1e13 cycles) -- such items are counted
    # and left out of every statistic below, as are items with 0 ADMM iterations
    ok = (ph_all >= 0).all(axis=1) & (ph_all < 5e8).all(axis=1) & (d[:, 9] > 0) & (d[:, 7] > d[:, 0])
    n_bad = int((~ok).sum())
    # In a fused launch an instance's items run on different workgroups, often on different XCDs: the slots then
    # may keep stamps of two different items (stores from different XCDs' L2s land in either order), and s_memtime
    # counts per XCD, so such a mix gives garbage differences.  Items whose sub-phase stamps are not one monotone
    # sequence are left out as well (counted).
    sub_idx = [1, 20, 21, 16, 17, 18, 19, 4] if fused else [1, 16, 17, 18, 19, 4]   # (20, 21: fused linearization)
    sd = np.diff(d[:, sub_idx], axis=1)
    ok_sub = ok & (sd >= 0).all(axis=1) & (sd < 5e8).all(axis=1)
    n_mix = int((ok & ~ok_sub).sum())
    ok = ok_sub
    d = d[ok]
    B = d.shape[0]
    ph = ph_all[ok]
    print(f"kernel {e0.elapsed_time(e1):.3f} ms  B={B + n_bad + n_mix} N={N} kind={kind} polish_mode={polish_mode}"
          f"  ({n_bad} items without an ADMM solve left out: solver error / infeasible up front; {n_mix} items"
          f" with stamps of two items, left out)")
    print("phase       median      p90       max   (cycles)")
    for i, nm in enumerate(names):
        print(f"{nm:10s} {np.median(ph[:, i]):9.0f} {np.percentile(ph[:, i], 90):9.0f} {ph[:, i].max():9.0f}")
    if fused:
        # slot 22: first-step start (indexed by workgroup), 23: last-step end (by instance), 100 MHz
        st0, en = d[:, 22].astype(float), d[:, 23].astype(float)
        t0 = st0.min()
        span = (en.max() - t0) / 100.0
        print("fused launch span %.1f us; workgroup starts: median %.1f p90 %.1f max %.1f us; instance ends: median %.1f"
              " p90 %.1f max %.1f us" % (span, np.median(st0 - t0) / 100, np.percentile(st0 - t0, 90) / 100,
                                         (st0.max() - t0) / 100, np.median(en - t0) / 100,
                                         np.percentile(en - t0, 90) / 100, (en.max() - t0) / 100))
        print("workgroups started within 20 us of the first: %d (resident capacity)" % int(((st0 - t0) < 2000).sum()))
        lin = np.diff(d[:, [1, 20, 21, 16]], axis=1)
        for i, nm in enumerate(["  rollout", "  jac state columns", "  jac phi/d/delta + g"]):
            print(f"{nm:22s} {np.median(lin[:, i]):9.0f} {np.percentile(lin[:, i], 90):9.0f}")
    sub = np.diff(d[:, [1, 16, 17, 18, 19, 4]], axis=1)
    for i, nm in enumerate(["  window/stage-issue", "  sincos+landed", "  stage loop", "  P rows", "  penalties"]):
        print(f"{nm:22s} {np.median(sub[:, i]):9.0f} {np.percentile(sub[:, i], 90):9.0f}")
    tot = d[:, 7] - d[:, 0]
    print(f"{'total':10s} {np.median(tot):9.0f} {np.percentile(tot, 90):9.0f} {tot.max():9.0f}")
    it, nf, ps = d[:, 9], d[:, 8], d[:, 10]
    print("iters median", np.median(it), "p99", np.percentile(it, 99), "max", it.max(), " factorizations median", np.median(nf), "max", nf.max())
    solve = ph[:, 3]
    A = np.stack([it, nf, np.ones_like(it)], 1).astype(float)
    coef, *_ = np.linalg.lstsq(A, solve.astype(float), rcond=None)
    print("solve cycles ~ %.0f/iter + %.0f/factorization + %.0f" % tuple(coef))
    res, sw, pol, nres = d[:, 11], d[:, 12], d[:, 13], d[:, 14]
    admm = solve - res - sw - pol
    print("solve split (median / sum share): residual checks %.0f / %.2f, sweeps %.0f / %.2f, polish %.0f / %.2f, ADMM iterations %.0f / %.2f"
          % (np.median(res), res.sum() / solve.sum(), np.median(sw), sw.sum() / solve.sum(), np.median(pol), pol.sum() / solve.sum(),
             np.median(admm), admm.sum() / solve.sum()))
    print("per residual check %.0f cycles, per sweep %.0f, per plain iteration %.0f"
          % (res.sum() / max(nres.sum(), 1), sw.sum() / max(nf.sum(), 1), admm.sum() / max(it.sum(), 1)))
    rs, re = d[:, 2] - d[:, 2].min(), d[:, 3] - d[:, 2].min()      # 100 MHz ticks
    print("wall (us): kernel span %.1f; starts: median %.1f max %.1f; ends: median %.1f p99 %.1f max %.1f"
          % (re.max() / 100, np.median(rs) / 100, rs.max() / 100, np.median(re) / 100, np.percentile(re, 99) / 100, re.max() / 100))
    last = np.argsort(re)[-5:]
    for b in last:
        print("  late finisher b=%d start %.1f us end %.1f us iters %d cycles %d" % (b, rs[b] / 100, re[b] / 100, it[b], tot[b]))
    clk = 0.1 * tot / np.maximum(re - rs, 1)
    print("in-kernel clock (median over instances): %.2f GHz" % np.median(clk))

if __name__ == "__main__":
    main(polish_mode=int(sys.argv[1]) if len(sys.argv) > 1 else 0, warm=int(sys.argv[2]) if len(sys.argv) > 2 else 5,
         fused=int(sys.argv[3]) if len(sys.argv) > 3 else 0, N=int(sys.argv[4]) if len(sys.argv) > 4 else 20,
         kind=sys.argv[5] if len(sys.argv) > 5 else "spline")
