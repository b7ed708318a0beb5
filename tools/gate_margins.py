"""Observed margins of the per-step oracle gates (diagnostics only; GPU + the C oracle in GPU-sine mode).

  python tools/gate_margins.py > gpurun_out/gate_margins.json

For each gate, every step of the GPU closed loop is re-solved by the step entry point and by the oracle from the
GPU's own state (as tests/test_config_sizes.py and tests/test_gpu_parity.py do), and the worst observed values of
the gated quantities are reported instead of asserted:
  * configs3_all: the configs[3] rank share (4096 spline, N = 20, dt 0.05, 240 steps) over all 4096 ids
    (tests/test_config_sizes.py's gate);
  * n40_ts005: test_closed_loop_per_step_parity_ts005[mixed-40-30-32-0].
Quantities: status mismatches, max |du| where both polished, max |du| where neither polished at the same ADMM
iteration (each with the (id, step) where it occurs and the ids above 1e-6), the fractions with equal polish
outcome and equal iteration counts."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def gate(TB, O, w, X, U, ids, N, Ts, T, chunk=1024):
    vr_all = np.tile(w["vref"], (len(w["x0"]), 1))
    cfg, ocfg = TB.config_struct(N=N, Ts=Ts), O.cfg(N=N, Ts=Ts)
    st = {"status_mismatch": 0, "du_both_max": 0.0, "du_eq_max": 0.0, "n": 0, "n_same_pol": 0, "n_same_it": 0}
    for t in range(T):
        for c0 in range(0, ids.size, chunk):
            sel0 = ids[c0:c0 + chunk]
            xt = X[sel0, t]
            ut = U[sel0, t - 1] if t > 0 else w["u0"][sel0]
            fin = np.isfinite(xt).all(axis=1) & np.isfinite(ut).all(axis=1)
            if not fin.any():
                continue
            sel, xt, ut = sel0[fin], xt[fin], ut[fin]
            pt = TB.PathSet.build(w["kinds"][sel], w["pcs"][sel], [w["knots"][i] for i in sel])
            prt = TB.ref_window_batch(pt, xt[:, 0], vr_all[sel], N, Ts).cpu().numpy()
            g = {k: v.cpu().numpy() for k, v in TB.mpc_step_batch(xt, ut, prt, vr_all[sel], cfg).items()}
            ro = O.mpc_step_batch(xt, ut, prt, vr_all[sel], ocfg)
            st["status_mismatch"] += int((g["status"] != ro["status"]).sum())
            ok = (g["status"] <= 1) & (g["status"] == ro["status"])
            du = np.abs(g["u_cmd"] - ro["u_cmd"]).max(axis=1)
            gp, rp = g["polished"] > 0, ro["polished"] > 0
            both = ok & gp & rp
            eq = ok & ~gp & ~rp & (g["iters"] == ro["iters"])
            for key, m in (("du_both", both), ("du_eq", eq)):
                v = float(du[m].max(initial=0.0))
                if v > st[key + "_max"]:
                    st[key + "_max"] = v
                    st[key + "_at"] = [int(sel[m][np.argmax(du[m])]), t]   # (id, step)
                # per-id worst, for the ids above 1e-6
                for i in sel[m & (du > 1e-6)]:
                    st.setdefault(key + "_ids_above_1e-6", {})
                    d = float(du[sel == i][0])
                    st[key + "_ids_above_1e-6"][str(int(i))] = max(st[key + "_ids_above_1e-6"].get(str(int(i)), 0.0), d)
            st["n"] += int(fin.sum())
            st["n_same_pol"] += int((gp == rp).sum())
            st["n_same_it"] += int((g["iters"] == ro["iters"]).sum())
    st["frac_same_pol"] = st["n_same_pol"] / max(st["n"], 1)
    st["frac_same_it"] = st["n_same_it"] / max(st["n"], 1)
    return st


def main():
    import oracle as O
    from trajectory_generation_amd import batch as TB
    from trajectory_generation_amd.workload import make_workload
    O.build()
    out = {}
    with O.tire_sine(1):
        t0 = time.time()
        B, T, N, Ts = 4096, 240, 20, 0.05
        w = make_workload(B, N, Ts, kind="spline", seed=0, id_offset=0)
        paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
        res = TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, TB.config_struct(N=N, Ts=Ts))
        X, U = res["X"].cpu().numpy(), res["U"].cpu().numpy()
        out["configs3_all"] = gate(TB, O, w, X, U, np.arange(B), N, Ts, T)
        out["configs3_all"]["seconds"] = time.time() - t0
        print(json.dumps({"configs3_all": out["configs3_all"]}), file=sys.stderr, flush=True)
        t0 = time.time()
        B, T, N, Ts = 32, 30, 40, 0.05
        w = make_workload(B, N, Ts, kind="mixed", seed=9)
        paths = TB.PathSet.build(w["kinds"], w["pcs"], w["knots"])
        res = TB.run_closed_loop(w["x0"], w["u0"], paths, w["vref"], T, TB.config_struct(N=N, Ts=Ts, warm_start=0))
        X, U = res["X"].cpu().numpy(), res["U"].cpu().numpy()
        out["n40_ts005"] = gate(TB, O, w, X, U, np.arange(B), N, Ts, T)
        out["n40_ts005"]["seconds"] = time.time() - t0
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
