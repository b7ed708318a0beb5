// mpc_long.h -- the MPC step for horizons past the register-resident kernels: TRAJ_MAX_N < N <= TRAJ_MAX_N_LONG,
// no state bounds (the reference's callers pass none; with state bounds every horizon runs mpc_general.h).
//
// Reference: MPC/mpc_6stati.py:120-275 (mpc_step takes any N, :125).  The algorithm is the hot kernel's
// (mpc_solve.h), restated for a matrix that no longer fits a wave's registers:
//   * the condensed QP over U (n = 2N variables), box + rate rows, so A stays bidiagonal: variable t owns its box
//     row and its rate row, and every product with A or A' is a +-2 neighbour exchange;
//   * OSQP 0.6's ADMM (Ruiz scaling with cost scaling, sigma / alpha, adaptive rho every check_interval iterations,
//     OSQP termination) and polish (mode 0: OSQP's reduced KKT + acceptance rule; mode 1: the exact active-set
//     polish with its KKT certificate), as the CPU oracle under oracle/ restates them;
//   * K = P + sigma I + A' diag(rho) A is inverted explicitly by the symmetric sweep operator (n pivots), so every
//     ADMM iteration is one dense mat-vec -- as in the hot kernel.
// CLOSED: one closed-loop step of MPC/main.py:85-101 (traj_closed_loop_step / _run past TRAJ_MAX_N): the state and
// u_prev from the closed-loop buffers, the reference window from the state (main.py:51-68, as mpc_solve.h does), the
// warm-start rho carried in the workspace's warm record, and the plant update x <- x + Ts f(x, u_cmd) (:97), u_prev
// <- u_cmd (:101) with the history, instead of X_opt / U_opt / the objective.
// Layout: one NT-thread workgroup per instance (NT = 256, or 512 past n = 256), thread t owns variable t (n <= NT).  The scaled P lives in the
// caller's scratch, COLUMN-major (entry (r, j) at j ld + r: for fixed j the threads read consecutive doubles), ld x ld
// with ld = n rounded up to 8 and zero padding; K^-1 the same way, in LDS (dynamic shared memory, n <= LONG_NKL:
// 128 KB at n = 128) or in the scratch beyond.  A pivot of the sweep, a mat-vec, a Ruiz pass each stream the
// matrix once through the workgroup, 8 columns at a time with the next 8 loaded before this 8 are stored (a row
// update is a read-modify-write whose columns the compiler cannot prove distinct, so without the explicit pipeline
// every load waits for the previous store); the vectors (broadcasts, +-2 exchanges, block maxima) go through small
// LDS buffers.
#pragma once
#include "mpc_common.h"

namespace tgmpc {

constexpr int LONG_NT = 256;                  // threads per instance = max n (n <= 256)
constexpr int LONG_NT2 = 512;                 // the instance for 256 < n <= 512 (round 6: N up to 256)
constexpr int LONG_NKL = 128;                 // n up to which K^-1 lives in LDS

__host__ __device__ inline int long_ld(int n) { return (n + 7) & ~7; }
// per-instance scratch (doubles): P, and K^-1 when it does not fit LDS
__host__ __device__ inline size_t long_ws_doubles(int N) {
    const int n = 2 * N, ld = long_ld(n);
    return (size_t)ld * ld * (n > LONG_NKL ? 2 : 1);
}
__host__ inline size_t long_lds_bytes(int N) {
    const int n = 2 * N;
    return n <= LONG_NKL ? (size_t)long_ld(n) * long_ld(n) * sizeof(double) : 0;
}

template <bool KL, bool CLOSED = false, int NT = LONG_NT>
__global__ __launch_bounds__(NT) void solve_long_kernel(const KArgs a, double* lws, size_t lstride) {
    extern __shared__ __attribute__((aligned(16))) double s_kl[];   // K^-1 (KL)
    __shared__ double s_bc[2][NT];       // broadcast vectors (rotating)
    __shared__ double s_ex[4][NT];       // +-2 exchanges (rotating)
    __shared__ double s_pc[NT];          // the sweep's pivot column
    __shared__ double s_xh[6];                // free response, one stage
    __shared__ double s_F[3][NT];        // condensing: F_k rows
    __shared__ double s_red[(NT / 64) * 8];
    __shared__ int s_flag[4];
    // CLOSED: the step's state, u_prev and reference window (main.py:51-68) -- x_state / u_state are overwritten by the
    // plant update at the end, so every read goes through these copies
    __shared__ double s_xc[CLOSED ? 6 : 1], s_uc[CLOSED ? 2 : 1], s_prc[CLOSED ? 3 * (NT / 2 + 1) : 1];
    const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const traj_vehicle_params& p = a.p;
    const traj_mpc_config& c = a.c;
    const int N = c.N, n = 2 * N, ld = long_ld(n);
    const bool own = t < n;
    const int kk = t >> 1, ch = t & 1;
    double* const P = lws + (size_t)b * lstride;                    // [j ld + r]
    double* const Kg = P + (size_t)ld * ld;                          // K^-1 in the scratch (!KL)
    auto Kat = [&](int j) -> double& {
        if constexpr (KL) return s_kl[j * ld + t];
        else return Kg[(size_t)j * ld + t];
    };
    auto Pat = [&](int j) -> double& { return P[(size_t)j * ld + t]; };
    // row t of a matrix (K or P), columns [0, jend) (jend a multiple of 8): v[j] <- f(j, v[j]), 8 columns at a time,
    // the next chunk loaded before this one is stored
    auto row_map = [&](auto&& at, int jend, auto&& f) {
        double cur[8], nxt[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) cur[i] = at(i);
        for (int j0 = 0; j0 < jend; j0 += 8) {
            if (j0 + 8 < jend) {
#pragma unroll
                for (int i = 0; i < 8; ++i) nxt[i] = at(j0 + 8 + i);
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) at(j0 + i) = f(j0 + i, cur[i]);
#pragma unroll
            for (int i = 0; i < 8; ++i) cur[i] = nxt[i];
        }
    };
    // sum_j row_t[j] v[j] (4 chains, the hot kernel's Kmul order) and max_j |row_t[j]|, 8 columns at a time
    auto row_dot = [&](auto&& at, const double* v) -> double {
        double s4[4] = {0.0, 0.0, 0.0, 0.0};
        for (int j0 = 0; j0 < ld; j0 += 8) {
            double kv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) kv[i] = at(j0 + i);
#pragma unroll
            for (int i = 0; i < 8; ++i) s4[i & 3] = fma(kv[i], v[j0 + i], s4[i & 3]);
        }
        return (s4[0] + s4[1]) + (s4[2] + s4[3]);
    };
    auto row_absmax = [&](auto&& at) -> double {
        double m = 0.0;
        for (int j0 = 0; j0 < ld; j0 += 8) {
            double kv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) kv[i] = at(j0 + i);
#pragma unroll
            for (int i = 0; i < 8; ++i) m = fmax(m, fabs(kv[i]));
        }
        return m;
    };
    const double* vr = a.vref + (size_t)(N + 1) * b;
    if constexpr (CLOSED) {
        if (t < 6) s_xc[t] = a.x_state[6 * (size_t)b + t];
        if (t < 2) s_uc[t] = a.u_state[2 * (size_t)b + t];
        __syncthreads();
        // main.py:51-68: xs_0 = X, xs_{k+1} = xs_k + vref_k Ts (serial, as ref_window_kernel / mpc_solve.h); ys = path(xs),
        // phi* = atan(path'(xs))
        if (t == 0) {
            double xs = s_xc[0];
            s_prc[0] = xs;
            for (int k = 0; k < N; ++k) {
                xs = xs + vr[k] * c.Ts;
                s_prc[3 * (k + 1)] = xs;
            }
        }
        __syncthreads();
        for (int k = t; k <= N; k += NT) {
            double y, dy;
            path_eval(a.path, b, s_prc[3 * k], y, dy);
            s_prc[3 * k + 1] = y;
            s_prc[3 * k + 2] = pm_atan(dy);
        }
        __syncthreads();
    }
    const double* x0 = CLOSED ? s_xc : a.x0 + 6 * (size_t)b;
    const double* up = CLOSED ? s_uc : a.u_prev + 2 * (size_t)b;
    const double* pref = CLOSED ? s_prc : a.path_ref + (size_t)3 * (N + 1) * b;
    const double* gA = a.Ad + (size_t)36 * N * b;
    const double* gB = a.Bd + (size_t)12 * N * b;
    const double* gg = a.gd + (size_t)6 * N * b;

    // ---- block helpers ----
    int xb = 0, bb = 0;
    auto exch = [&](double v, int delta) -> double {   // value of variable t + delta (0 outside 0..n-1)
        double* buf = s_ex[xb & 3];
        xb++;
        buf[t] = v;
        __syncthreads();
        const int s = t + delta;
        return (own && s >= 0 && s < n) ? buf[s] : 0.0;
    };
    auto bcast = [&](double v) -> const double* {
        double* buf = s_bc[bb & 1];
        bb++;
        buf[t] = own ? v : 0.0;
        __syncthreads();
        return buf;
    };
    // block max of V values, NaN propagating (uniform result)
    auto block_max = [&](auto& v) {
        constexpr int V = sizeof(v) / sizeof(double);
        static_assert(V <= 8, "s_red");
        bool nan[V];
#pragma unroll
        for (int i = 0; i < V; ++i) {
            nan[i] = __syncthreads_or(v[i] != v[i]);
            double m = v[i] != v[i] ? 0.0 : v[i];
            for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
            if (lane == 0) s_red[wid * 8 + i] = m;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < V; ++i) {
            double m = s_red[i];
            for (int w = 1; w < NT / 64; ++w) m = fmax(m, s_red[w * 8 + i]);
            v[i] = nan[i] ? __builtin_nan("") : m;
        }
        __syncthreads();
    };
    // block sum in a fixed order (wave partials in lane order, then waves in order)
    auto block_sum = [&](double v) -> double {
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) s_red[wid * 8] = v;
        __syncthreads();
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += s_red[w * 8];
        __syncthreads();
        return s;
    };

    // ---- inputs (:144-163 normalisation done by the caller) ----
    if (t == 0) { s_flag[0] = 0; s_flag[1] = 0; }
    __syncthreads();
    {
        int bad = 0;
        if (t < 6) bad |= !isfinite(x0[t]);
        if (t < 2) bad |= !isfinite(up[t]);
        for (int i = t; i < 3 * (N + 1); i += NT) bad |= !isfinite(pref[i]);
        for (int i = t; i < N + 1; i += NT) bad |= !isfinite(vr[i]);
        if (bad) s_flag[0] = 1;
    }

    // ---- condensed QP (:180-250): P = sum_k F_k' F_k (+ the input penalties), q ----
    // thread t carries column t of the input sensitivity G_k; the free response xh is uniform
    const double sw0 = sqrt(2.0 * c.q_c), sw1 = sqrt(2.0 * c.q_phi), sw2 = sqrt(2.0 * c.q_vx);
    double xh[6], G[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 6; ++i) xh[i] = x0[i];
    double qi = 0.0;
    if (own)
        for (int j = 0; j < ld; ++j) Pat(j) = 0.0;
    for (int k = 0; k < N; ++k) {
        const double* Ak = gA + 36 * k;
        double xn[6], Gn[6];
        for (int r = 0; r < 6; ++r) {
            double v = gg[6 * k + r], w = 0.0;
            for (int cc = 0; cc < 6; ++cc) {
                v = fma(Ak[6 * r + cc], xh[cc], v);
                w = fma(Ak[6 * r + cc], G[cc], w);
            }
            xn[r] = v;
            Gn[r] = (own && kk == k) ? gB[12 * k + 2 * r + ch] : w;
        }
        for (int r = 0; r < 6; ++r) { xh[r] = xn[r]; G[r] = Gn[r]; }
        const int k1 = k + 1;
        double sk, ck;
        pm_sincos(pref[3 * k1 + 2], &sk, &ck);
        const double e0 = sk * (xh[0] - pref[3 * k1]) - ck * (xh[1] - pref[3 * k1 + 1]);
        const double e1 = xh[2] - pref[3 * k1 + 2];
        const double e2 = xh[3] - vr[k1];
        const double F0 = sw0 * (sk * G[0] - ck * G[1]), F1 = sw1 * G[2], F2 = sw2 * G[3];
        qi += sw0 * F0 * e0 + sw1 * F1 * e1 + sw2 * F2 * e2;
        s_F[0][t] = F0; s_F[1][t] = F1; s_F[2][t] = F2;
        __syncthreads();
        // F_k's columns >= 2 (k + 1) are zero (the inputs of later stages): row t's entries j < 2 k + 2 only (to the
        // next multiple of 8; threads >= n hold F = 0, so the padding columns stay zero)
        if (own) {
            const int jm = 2 * k + 2 < n ? 2 * k + 2 : n;
            row_map(Pat, (jm + 7) & ~7, [&](int j, double v) {
                return fma(F0, s_F[0][j], fma(F1, s_F[1][j], fma(F2, s_F[2][j], v)));
            });
        }
        __syncthreads();
    }
    // input penalties U'RU and dU'Rd dU (dU_0 = U_0 - u_prev): the band of row t
    double Rs[4], Rds[4];
    Rs[0] = c.R[0]; Rs[3] = c.R[3]; Rs[1] = Rs[2] = 0.5 * (c.R[1] + c.R[2]);
    Rds[0] = c.Rd[0]; Rds[3] = c.Rd[3]; Rds[1] = Rds[2] = 0.5 * (c.Rd[1] + c.Rd[2]);
    const double Rs0 = ch ? Rs[2] : Rs[0], Rs1 = ch ? Rs[3] : Rs[1];
    const double Rd0 = ch ? Rds[2] : Rds[0], Rd1 = ch ? Rds[3] : Rds[1];
    const double dmul = (kk < N - 1) ? 2.0 : 1.0;
    if (own) {
        const int j0 = 2 * kk - 2 > 0 ? 2 * kk - 2 : 0, j1 = 2 * kk + 4 < n ? 2 * kk + 4 : n;
        for (int j = j0; j < j1; ++j) {
            const int kj = j >> 1;
            const double rs = (j & 1) ? Rs1 : Rs0, rd = (j & 1) ? Rd1 : Rd0;
            double add = (kj == kk) ? 2.0 * rs + 2.0 * rd * dmul : 0.0;
            add = (kj == kk - 1 || kj == kk + 1) ? -2.0 * rd : add;
            Pat(j) += add;
        }
        if (kk == 0) qi -= 2.0 * (Rd0 * up[0] + Rd1 * up[1]);
    }
    // constraint rows owned by t: box (U_t) and rate (U_t - U_{t-2}, or U_0 - u_prev)
    double lb = ch ? c.u_lo[1] : c.u_lo[0], ub = ch ? c.u_hi[1] : c.u_hi[0];
    double lr = ch ? c.du_lo[1] : c.du_lo[0], ur = ch ? c.du_hi[1] : c.du_hi[0];
    if (kk == 0) { lr += up[ch]; ur += up[ch]; }
    const bool has_prev = kk > 0;
    {
        int bad = 0;
        if (own) {
            bad |= !isfinite(qi);
            bad |= !isfinite(row_absmax(Pat));
        }
        if (bad) s_flag[0] = 1;
    }
    // exact feasibility of the box + rate chain (interval propagation)
    if (t < 2) {
        double lo = up[t], hi = up[t];
        const double dlo = t ? c.du_lo[1] : c.du_lo[0], dhi = t ? c.du_hi[1] : c.du_hi[0];
        const double ulo = t ? c.u_lo[1] : c.u_lo[0], uhi = t ? c.u_hi[1] : c.u_hi[0];
        for (int k = 0; k < N; ++k) {
            double nlo = lo + dlo, nhi = hi + dhi;
            if (nlo < ulo) nlo = ulo;
            if (nhi > uhi) nhi = uhi;
            if (!(nlo <= nhi)) s_flag[1] = 1;
            lo = nlo;
            hi = nhi;
        }
    }
    __syncthreads();
    const int early = s_flag[0] ? TRAJ_STATUS_SOLVER_ERROR : (s_flag[1] ? TRAJ_STATUS_INFEASIBLE : -1);
    int status = TRAJ_STATUS_SOLVER_ERROR, iter = 0, pol = 0;
    double xsol = 0.0;

    if (early < 0) {
        // ---- Ruiz equilibration + cost scaling (OSQP scale_data), as mpc_solve.h ----
        double D = 1.0, Eb = 1.0, Er = 1.0, cs = 1.0, cn = 0.0;
        if (own)
            cn = row_absmax(Pat);
        for (int it = 0; it < c.scaling_iters; ++it) {
            const double Er_up = exch(Er, +2), D_dn = exch(D, -2);
            const double a_b = Eb * D, a_r = Er * D, a_rm = has_prev ? Er * D_dn : 0.0, a_rp = Er_up * D;
            const double pn = cs * cn;
            const double coln = fmax(pn, fmax(fmax(fabs(a_b), fabs(a_r)), fabs(a_rp)));
            const double Dt = own ? 1.0 / sqrt(limit_scaling(coln)) : 1.0;
            const double Etb = 1.0 / sqrt(limit_scaling(fabs(a_b)));
            const double Etr = 1.0 / sqrt(limit_scaling(fmax(fabs(a_r), fabs(a_rm))));
            const double* dv = bcast(Dt);
            cn = 0.0;
            if (own)
                row_map(Pat, ld, [&](int j, double v) {
                    const double w = v * (Dt * dv[j]);
                    cn = fmax(cn, fabs(w));
                    return w;
                });
            qi *= Dt;
            D *= Dt;
            Eb *= Etb;
            Er *= Etr;
            const double mean = block_sum(own ? cs * cn : 0.0) / n;
            double qv[1] = {own ? fabs(cs * qi) : 0.0};
            block_max(qv);
            double ct = fmax(mean, limit_scaling(qv[0]));
            ct = 1.0 / limit_scaling(ct);
            cs *= ct;
        }
        if (own) row_map(Pat, ld, [&](int, double v) { return v * cs; });
        qi *= cs;
        const double csinv = 1.0 / cs;
        const double D_dn = exch(D, -2);
        const double a_b = Eb * D, a_r = Er * D, a_rm = has_prev ? Er * D_dn : 0.0;
        const double a_r_up = exch(a_r, +2);
        const double slb = (lb > -INFTY) ? lb * Eb : -INFTY, sub = (ub < INFTY) ? ub * Eb : INFTY;
        const double slr = (lr > -INFTY) ? lr * Er : -INFTY, sur = (ur < INFTY) ? ur * Er : INFTY;
        const double Dinv = 1.0 / D, Ebinv = 1.0 / Eb, Erinv = 1.0 / Er;
        __syncthreads();   // P scaled (the mat-vecs below read other threads' rows by column)

        // ---- helpers over the scaled problem ----
        auto Ax = [&](double v, double& zb, double& zr) {
            const double vdn = exch(v, -2);
            zb = a_b * v;
            zr = a_r * v - a_rm * vdn;
        };
        auto ATw = [&](double wb, double wr) -> double {
            const double rp_up = exch(a_rm * wr, +2);   // a_rp(t) wr(t+2), formed on thread t+2
            return a_b * wb + a_r * wr - rp_up;
        };
        auto Pmul = [&](double v) -> double {   // (P v)_t, P symmetric: row t = column t
            const double* vb = bcast(v);
            return own ? row_dot(Pat, vb) : 0.0;
        };
        auto Kmul = [&](double v) -> double {   // (K^-1 v)_t
            const double* vb = bcast(v);
            return own ? row_dot(Kat, vb) : 0.0;
        };
        auto rho_for = [&](double l, double u, double rho) -> double {
            if (l <= -INFTY * MIN_SCALING && u >= INFTY * MIN_SCALING) return RHO_MIN;
            if (u - l < RHO_TOL) return RHO_EQ_OVER_INEQ * rho;
            return rho;
        };
        struct Res { double pr, dr, eps_p, eps_d, prs, drs, pn, dn; };
        auto residuals = [&](double x, double zb, double zr, double yb, double yr) -> Res {
            const double px = Pmul(x);
            double axb, axr;
            Ax(x, axb, axr);
            const double aty = ATw(yb, yr);
            double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (own) {
                const double dres = px + qi + aty;
                v[0] = fmax(fabs(Ebinv * (axb - zb)), fabs(Erinv * (axr - zr)));
                v[1] = fmax(fmax(fabs(Ebinv * axb), fabs(Erinv * axr)), fmax(fabs(Ebinv * zb), fabs(Erinv * zr)));
                v[2] = fabs(Dinv * dres) * csinv;
                v[3] = fmax(fabs(Dinv * px) * csinv, fmax(fabs(Dinv * aty) * csinv, fabs(Dinv * qi) * csinv));
                v[4] = fmax(fabs(axb - zb), fabs(axr - zr));
                v[5] = fabs(dres);
                v[6] = fmax(fmax(fabs(axb), fabs(axr)), fmax(fabs(zb), fabs(zr)));
                v[7] = fmax(fmax(fabs(aty), fabs(qi)), fabs(px));
            }
            block_max(v);
            Res r;
            r.pr = v[0]; r.eps_p = c.eps_abs + c.eps_rel * v[1];
            r.dr = v[2]; r.eps_d = c.eps_abs + c.eps_rel * v[3];
            r.prs = v[4]; r.drs = v[5]; r.pn = v[6]; r.dn = v[7];
            return r;
        };

        // ---- ADMM (osqp_solve) + polish around one factorization site (mpc_solve.h's state machine) ----
        constexpr int PH_ADMM = 0, PH_POLISH = 1, PH_DONE = 2;
        int phase = PH_ADMM;
        double rho = c.rho;
        // closed-loop warm start (t > 0): the rho the instance's previous step adapted to (mpc_solve.h, the oracle's
        // orc_warm); iterates start at zero as cold
        if (CLOSED && c.warm_start && a.t > 0 && a.wsWarm) {
            const double* wv = a.wsWarm + 4 * (size_t)b;
            if (wv[1] != 0.0) rho = fmin(fmax(wv[0], RHO_MIN), RHO_MAX);
        }
        double x = 0.0, zb = 0.0, zr = 0.0, yb = 0.0, yr = 0.0;
        double rb = rho_for(slb, sub, rho), rr = rho_for(slr, sur, rho);
        Res r = {0, 0, 0, 0, 0, 0, 0, 0};
        int rounds = 0, ps = 0, actb = 0, actr = 0;
        double escale = 1.0;
        const double alpha = c.alpha, sig = c.sigma, dl = c.delta;
        iter = 1;
        while (phase != PH_DONE) {
            // ---- K = P + ks I + A' diag(kb, kr) A, then the sweep: K <- -K^-1 ----
            const double kb = (phase == PH_ADMM) ? rb : (actb ? 1.0 / dl : 0.0);
            const double kr = (phase == PH_ADMM) ? rr : (actr ? 1.0 / dl : 0.0);
            const double ks = (phase == PH_ADMM) ? sig : dl;
            {
                const double kr_up = exch(kr, +2);
                const double a_rp = exch(a_rm, +2);   // Er(t+2) D(t)
                const double dii = ks + kb * a_b * a_b + kr * a_r * a_r + kr_up * a_rp * a_rp;
                const double dp = -kr_up * a_r_up * a_rp;          // (t, t+2)
                const double dm = -kr * a_r * a_rm;                // (t, t-2): thread t-2's dp, the same product
                if (own)
                    for (int j0 = 0; j0 < ld; j0 += 8) {
                        double v[8];
#pragma unroll
                        for (int i = 0; i < 8; ++i) v[i] = Pat(j0 + i);
#pragma unroll
                        for (int i = 0; i < 8; ++i) {
                            const int j = j0 + i;
                            double w = v[i];
                            w = (j == t) ? w + dii : w;
                            w = (j == t + 2) ? w + dp : w;
                            w = (j == t - 2 && has_prev) ? w + dm : w;
                            Kat(j) = w;
                        }
                    }
            }
            bool ok = true;
            for (int pv = 0; pv < n; ++pv) {
                __syncthreads();
                s_pc[t] = own ? Kat(pv) : 0.0;   // (rows >= n: zero, so the padding columns stay zero)
                __syncthreads();
                const double d = s_pc[pv];
                ok = ok && (d > 0.0);
                const double dinv = 1.0 / d;
                if (own) {
                    const bool piv = t == pv;
                    const double fd = s_pc[t] * dinv;
                    const double be = piv ? dinv : -fd;
                    const double al = piv ? 0.0 : 1.0;
                    row_map(Kat, ld, [&](int j, double v) { return fma(be, s_pc[j], al * v); });
                    Kat(pv) = piv ? -dinv : fd;
                }
            }
            __syncthreads();
            if (own) row_map(Kat, ld, [&](int, double v) { return -v; });
            __syncthreads();
            if (!ok) {
                if (phase == PH_ADMM) { status = TRAJ_STATUS_SOLVER_ERROR; break; }
                if (c.polish_mode == 1 && rounds < c.polish_max_rounds && iter < c.max_iter) {
                    ++rounds;
                    escale *= 1e-2;
                    ++iter;
                    phase = PH_ADMM;
                } else {
                    phase = PH_DONE;
                }
                continue;
            }
            if (phase == PH_ADMM) {
                bool converged = false, refactor = false;
                int chk = c.check_interval - (iter - 1) % c.check_interval;
                const double oma = 1.0 - alpha;
                const double rib = 1.0 / rb, rir = 1.0 / rr;
                for (; iter <= c.max_iter; ++iter) {
                    const double wb = fma(rb, zb, -yb), wr = fma(rr, zr, -yr);
                    const double rp_up = exch(a_rm * wr, +2);
                    const double atw = fma(a_b, wb, fma(a_r, wr, -rp_up));
                    const double xt = Kmul(fma(sig, x, atw - qi));
                    const double xt_dn = exch(xt, -2);
                    const double ztb = a_b * xt, ztr = fma(a_r, xt, -(a_rm * xt_dn));
                    const double xn = fma(alpha, xt, oma * x);
                    const double zrb = fma(alpha, ztb, oma * zb), zrr = fma(alpha, ztr, oma * zr);
                    const double nzb = clamp_mm(fma(rib, yb, zrb), slb, sub), nzr = clamp_mm(fma(rir, yr, zrr), slr, sur);
                    yb = fma(rb, zrb - nzb, yb);
                    yr = fma(rr, zrr - nzr, yr);
                    x = xn;
                    zb = nzb;
                    zr = nzr;
                    if (--chk == 0) {
                        chk = c.check_interval;
                        r = residuals(x, zb, zr, yb, yr);
                        if (r.pr <= escale * r.eps_p && r.dr <= escale * r.eps_d) { converged = true; break; }
                        if (c.adaptive_rho) {
                            double est = rho * sqrt((r.prs / (r.pn + DIV_TOL)) / (r.drs / (r.dn + DIV_TOL) + DIV_TOL));
                            est = fmin(fmax(est, RHO_MIN), RHO_MAX);
                            if (est > rho * c.adaptive_rho_tol || est < rho / c.adaptive_rho_tol) {
                                rho = est;
                                rb = rho_for(slb, sub, rho);
                                rr = rho_for(slr, sur, rho);
                                refactor = true;
                                ++iter;
                                break;
                            }
                        }
                    }
                }
                if (refactor && iter <= c.max_iter) continue;
                if (converged) status = TRAJ_STATUS_OPTIMAL;
                else {
                    iter = c.max_iter;
                    r = residuals(x, zb, zr, yb, yr);
                    status = (rounds > 0 && r.pr <= r.eps_p && r.dr <= r.eps_d) ? TRAJ_STATUS_OPTIMAL
                             : (r.pr <= 10.0 * r.eps_p && r.dr <= 10.0 * r.eps_d) ? TRAJ_STATUS_OPTIMAL_INACCURATE
                                                                                 : TRAJ_STATUS_USER_LIMIT;
                }
                if (status == TRAJ_STATUS_OPTIMAL && c.polish) {
                    // OSQP active sets: lower if z - l < -y, upper if u - z < y
                    actb = own ? ((zb - slb < -yb) ? -1 : ((sub - zb < yb) ? 1 : 0)) : 0;
                    actr = own ? ((zr - slr < -yr) ? -1 : ((sur - zr < yr) ? 1 : 0)) : 0;
                    ps = 1;
                    phase = PH_POLISH;
                } else {
                    phase = PH_DONE;
                }
                continue;
            }
            // ---- polish: K^-1 = M^-1, M = P + delta I + Ar' Ar / delta (the eliminated reduced KKT) ----
            {
                const double bbv = actb < 0 ? slb : (actb > 0 ? sub : 0.0);
                const double brv = actr < 0 ? slr : (actr > 0 ? sur : 0.0);
                double px_ = 0.0, pyb = 0.0, pyr = 0.0;
                double r1 = -qi, r2b = actb ? bbv : 0.0, r2r = actr ? brv : 0.0;
                double axb = 0.0, axr = 0.0;
                for (int rf = 0; rf <= c.polish_refine_iter; ++rf) {
                    const double tv = Kmul(r1 + ATw(actb ? r2b / dl : 0.0, actr ? r2r / dl : 0.0));
                    double tb, tr;
                    Ax(tv, tb, tr);
                    px_ += tv;
                    if (actb) pyb += (tb - r2b) / dl;
                    if (actr) pyr += (tr - r2r) / dl;
                    if (rf == c.polish_refine_iter) break;
                    const double Pxv = Pmul(px_);
                    const double atyv = ATw(pyb, pyr);
                    r1 = -qi - Pxv - atyv;
                    Ax(px_, axb, axr);
                    r2b = actb ? bbv - axb : 0.0;
                    r2r = actr ? brv - axr : 0.0;
                }
                Ax(px_, axb, axr);
                if (c.polish_mode == 0) {
                    // z = proj(Ax + y), y = Ax + y - z (OSQP project_normalcone); accept if the residuals drop
                    const double ztb = axb + pyb, ztr = axr + pyr;
                    const double nzb = clampd(ztb, slb, sub), nzr = clampd(ztr, slr, sur);
                    const double nyb = ztb - nzb, nyr = ztr - nzr;
                    const Res rp = residuals(px_, nzb, nzr, nyb, nyr);
                    const bool okp = (rp.pr < r.pr && rp.dr < r.dr) || (rp.pr < r.pr && r.dr < 1e-10) ||
                                     (rp.dr < r.dr && r.pr < 1e-10);
                    if (okp) {
                        x = px_; zb = nzb; zr = nzr; yb = nyb; yr = nyr;
                        pol = 1;
                    }
                    phase = PH_DONE;
                    continue;
                }
                // exact mode: the KKT certificate in the unscaled problem
                const double Pxv = Pmul(px_);
                const double atyv = ATw(pyb, pyr);
                const double tol = c.cert_tol;
                double v[2];
                double lb_ = ch ? c.u_lo[1] : c.u_lo[0], ub_ = ch ? c.u_hi[1] : c.u_hi[0];
                double lr_ = ch ? c.du_lo[1] : c.du_lo[0], ur_ = ch ? c.du_hi[1] : c.du_hi[0];
                if (kk == 0) { lr_ += up[ch]; ur_ += up[ch]; }
                v[0] = own ? fabs(Dinv * (Pxv + qi + atyv)) * csinv : 0.0;            // stationarity
                v[1] = own ? fmax(fabs(Dinv * qi), fabs(Dinv * Pxv)) * csinv : 0.0;  // gradient scale
                block_max(v);
                const double gsc = fmax(1.0, v[1]);
                int okc = v[0] <= tol * gsc;
                if (own) {
                    const double axu = axb * Ebinv, arv = axr * Erinv;
                    if (slb > -INFTY && axu < lb_ - tol * (1.0 + fabs(lb_))) okc = 0;
                    if (sub < INFTY && axu > ub_ + tol * (1.0 + fabs(ub_))) okc = 0;
                    if (slr > -INFTY && arv < lr_ - tol * (1.0 + fabs(lr_))) okc = 0;
                    if (sur < INFTY && arv > ur_ + tol * (1.0 + fabs(ur_))) okc = 0;
                    const double ybu = pyb * Eb * csinv, yru = pyr * Er * csinv;
                    if (actb < 0 && ybu > tol * gsc) okc = 0;
                    if (actb > 0 && ybu < -tol * gsc) okc = 0;
                    if (actr < 0 && yru > tol * gsc) okc = 0;
                    if (actr > 0 && yru < -tol * gsc) okc = 0;
                }
                double fo[1] = {okc ? 0.0 : 1.0};
                block_max(fo);
                if (fo[0] == 0.0) {
                    x = px_;
                    zb = clampd(axb, slb, sub);
                    zr = clampd(axr, slr, sur);
                    yb = pyb;
                    yr = pyr;
                    pol = ps + 16 * rounds;
                    phase = PH_DONE;
                    continue;
                }
                if (ps < c.polish_max_pass) {
                    // primal-dual active-set update with the OSQP rule on the polished (Ax, y)
                    actb = own ? ((axb - slb < -pyb) ? -1 : ((sub - axb < pyb) ? 1 : 0)) : 0;
                    actr = own ? ((axr - slr < -pyr) ? -1 : ((sur - axr < pyr) ? 1 : 0)) : 0;
                    ++ps;
                    continue;
                }
                if (rounds < c.polish_max_rounds && iter < c.max_iter) {
                    // not certified: continue ADMM to a 100x tighter tolerance, then polish again
                    ++rounds;
                    escale *= 1e-2;
                    ++iter;
                    phase = PH_ADMM;
                    continue;
                }
                phase = PH_DONE;
            }
        }
        if (iter > c.max_iter) iter = c.max_iter;
        xsol = D * x;
        if (CLOSED && a.wsWarm && t == 0) {
            double* wv = a.wsWarm + 4 * (size_t)b;
            wv[0] = rho;
            wv[1] = (status == TRAJ_STATUS_OPTIMAL || status == TRAJ_STATUS_OPTIMAL_INACCURATE) ? 1.0 : 0.0;
            wv[2] = (double)iter;
        }
    } else {
        status = early;
        iter = 0;
        if (CLOSED && a.wsWarm && t == 0) {
            a.wsWarm[4 * (size_t)b + 1] = 0.0;
            a.wsWarm[4 * (size_t)b + 2] = 0.0;
        }
    }

    // ---- outputs (:257-275): U, X_opt by the linear model, the objective, u_cmd ----
    const bool good = (status == TRAJ_STATUS_OPTIMAL || status == TRAJ_STATUS_OPTIMAL_INACCURATE);
    const double nan = __builtin_nan("");
    double* const Ub = s_bc[0];
    __syncthreads();
    Ub[t] = own ? xsol : 0.0;
    if (t < 6) s_xh[t] = x0[t];
    __syncthreads();
    if constexpr (CLOSED) {
        // plant x <- x + Ts f(x, u_cmd) (main.py:97), u_prev <- u_cmd (:101); the history and this step's outcome
        // (main.py:94 keeps only u_cmd: no X_opt, no objective)
        if (t == 0) {
            const double uc0 = good ? Ub[0] : up[0], uc1 = good ? Ub[1] : up[1];
            double xs[6], f[6], u[2] = {uc0, uc1};
            for (int i = 0; i < 6; ++i) xs[i] = x0[i];
            f_cont(p, xs, u, f);
            for (int i = 0; i < 6; ++i) {
                const double xn = xs[i] + c.Ts * f[i];
                a.x_state[6 * (size_t)b + i] = xn;
                if (a.hist_x) a.hist_x[((size_t)b * (a.hist_T + 1) + a.t + 1) * 6 + i] = xn;
            }
            a.u_state[2 * (size_t)b] = uc0;
            a.u_state[2 * (size_t)b + 1] = uc1;
            if (a.hist_u) {
                a.hist_u[((size_t)b * a.hist_T + a.t) * 2] = uc0;
                a.hist_u[((size_t)b * a.hist_T + a.t) * 2 + 1] = uc1;
            }
            if (a.status) a.status[b] = status;
            if (a.iters) a.iters[b] = iter;
        }
        return;
    }
    // X_{k+1} = A_k X_k + B_k U_k + g_k, stage by stage (thread r < 6: state r); X in s_ex (6 (N+1) <= 4 NT)
    double* const Xs = &s_ex[0][0];
    if (t < 6) Xs[t] = x0[t];
    __syncthreads();
    for (int k = 0; k < N; ++k) {
        if (t < 6) {
            double v = 0.0;
            for (int cc = 0; cc < 6; ++cc) v += gA[k * 36 + t * 6 + cc] * Xs[6 * k + cc];
            v += gB[k * 12 + t * 2] * Ub[2 * k] + gB[k * 12 + t * 2 + 1] * Ub[2 * k + 1] + gg[6 * k + t];
            Xs[6 * (k + 1) + t] = v;
        }
        __syncthreads();
    }
    double op = 0.0;
    for (int k = t; k <= N; k += NT) {
        const double* X = Xs + 6 * k;
        double s, co;
        pm_sincos(pref[3 * k + 2], &s, &co);
        const double ec = s * (X[0] - pref[3 * k]) - co * (X[1] - pref[3 * k + 1]);
        const double ep = X[2] - pref[3 * k + 2];
        const double ev = X[3] - vr[k];
        op += c.q_c * ec * ec + c.q_phi * ep * ep + c.q_vx * ev * ev;
        if (k < N) {
            const double u0 = Ub[2 * k], u1 = Ub[2 * k + 1];
            const double d0 = u0 - (k == 0 ? up[0] : Ub[2 * k - 2]);
            const double d1 = u1 - (k == 0 ? up[1] : Ub[2 * k - 1]);
            op += u0 * (c.R[0] * u0 + c.R[1] * u1) + u1 * (c.R[2] * u0 + c.R[3] * u1);
            op += d0 * (c.Rd[0] * d0 + c.Rd[1] * d1) + d1 * (c.Rd[2] * d0 + c.Rd[3] * d1);
        }
    }
    const double obj = block_sum(op);
    if (t == 0) {
        a.u_cmd[2 * b] = good ? Ub[0] : up[0];
        a.u_cmd[2 * b + 1] = good ? Ub[1] : up[1];
        a.status[b] = status;
        if (a.objective) a.objective[b] = good ? obj : nan;
        if (a.iters) a.iters[b] = iter;
        if (a.polished) a.polished[b] = pol;
    }
    if (a.U_opt && own) a.U_opt[(size_t)b * 2 * N + ch * N + kk] = good ? xsol : nan;
    if (a.X_opt)
        for (int i = t; i < 6 * (N + 1); i += NT) {
            const int rr = i / (N + 1), k = i % (N + 1);
            a.X_opt[(size_t)b * 6 * (N + 1) + i] = good ? Xs[6 * k + rr] : nan;
        }
}

}  // namespace tgmpc
