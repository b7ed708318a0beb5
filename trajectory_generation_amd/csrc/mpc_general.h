// mpc_general.h -- the MPC step's QP WITH optional state bounds (mpc_6stati.py:208-213) on the GPU.
//
// The hot kernel (mpc_solve.h) is specialised to the box + rate rows the reference's callers use:
// each QP variable owns its two rows and the constraint matrix is bidiagonal.  State bounds add
// 6 (N+1) rows X_k >= x_lo / X_k <= x_hi that are DENSE in the condensed variables
// (X_k = xh_k + G_k U), so this kernel solves the general condensed problem
//     min 1/2 U'PU + q'U  s.t.  l <= A U <= u,   A = [box | rate | state rows]  (m = 4N + nsr N rows)
// with the same OSQP restatement the C oracle under oracle/ runs (build_qp, osqp_scale,
// set_rho_vec, factor_kkt, residuals, primal_infeasible, kkt_solve_active, osqp_polish,
// exact_polish, osqp_solve, orc_mpc_step_warm), statement for statement:
//   * every reduction the oracle writes as a sequential loop is computed by one thread in the same
//     order (mat-vecs: one thread per output; sums: one thread), so the arithmetic is the oracle's;
//   * the Cholesky factorisation is right-looking over the workgroup -- entry (i, c) receives its
//     subtractions L[i][j] L[c][j] in increasing j, exactly the oracle's left-looking dot;
//   * the triangular solves run on one wave, column-oriented: row i's terms arrive in the order the
//     oracle's chol_solve adds them (ascending k forward, descending k backward);
//   * -ffp-contract=off on both sides; division and sqrt are IEEE-rounded.
// Layout: one 256-thread workgroup per instance; the Cholesky factor lives in LDS (n <= 80:
// 51 KB) or, for the horizons past the hot kernels' capacity (TRAJ_MAX_N < N <= TRAJ_MAX_N_GENERAL), in the
// caller's scratch; everything else in the caller's workspace: traj_mpc_sb_workspace_bytes(B, N) bytes past the
// step's workspace (traj_mpc_step_batch) or the workspace argument of traj_mpc_qp_batch (the library never
// allocates).  This path is for the optional argument and the long horizons only -- correctness first;
// the 4096-trajectory closed loop never takes it.
#pragma once
#include "mpc_common.h"

namespace tgmpc {

constexpr int GEN_NT = 256;
constexpr int GEN_NMAX = 2 * TRAJ_MAX_N;                    // n whose Cholesky factor is kept in LDS
// rows per lane of the one-wave triangular solves (a register array): the kernel is instantiated for n <= 512 (8 rows
// per lane, every horizon up to N = 256) and for n <= 2 TRAJ_MAX_N_GENERAL (launch_general picks by n)
constexpr int GEN_RMAX_SMALL = 8;
constexpr int GEN_RMAX = (2 * TRAJ_MAX_N_GENERAL + 63) / 64;
static_assert(GEN_RMAX >= GEN_RMAX_SMALL, "two instances");

// per-instance scratch of solve_gen_kernel, in doubles (m <= 10 N rows; n > GEN_NMAX: + the n x n factor)
__host__ __device__ inline size_t gen_ws_doubles(int N) {
    const size_t n = 2 * (size_t)N, m = 10 * (size_t)N;
    return n * n + m * n + 6 * (size_t)(N + 1) * n + 6 * (size_t)(N + 1) + 3 * n + 20 * n + 24 * m + 64 +
           (n > (size_t)GEN_NMAX ? n * n : 0);
}

struct GenWs {
    double *L;   // the Cholesky factor when it does not fit LDS (n > GEN_NMAX), else null
    double *P, *A, *G, *xh, *F;
    double *q, *D, *Dinv, *Dt, *x, *xt, *xp, *rhs, *Px, *Aty, *xpol, *r1, *tt, *xs, *U;   // n
    double *l, *u, *E, *Einv, *Et, *rv, *ri, *z, *y, *zt, *zp, *yp, *tm2, *Ax, *zpol, *ypol, *bb, *r2, *dd,
        *act, *rvp;   // m
};

__device__ inline GenWs gen_carve(double* p, int N) {
    const size_t n = 2 * (size_t)N, m = 10 * (size_t)N;
    GenWs w;
    auto take = [&](size_t k) {
        double* r = p;
        p += k;
        return r;
    };
    w.P = take(n * n);
    w.A = take(m * n);
    w.G = take(6 * (size_t)(N + 1) * n);
    w.xh = take(6 * (size_t)(N + 1));
    w.F = take(3 * n);
    double** vn[] = {&w.q, &w.D, &w.Dinv, &w.Dt, &w.x, &w.xt, &w.xp, &w.rhs, &w.Px, &w.Aty, &w.xpol, &w.r1, &w.tt,
                     &w.xs, &w.U};
    for (double** v : vn) *v = take(n);
    double** vm[] = {&w.l, &w.u, &w.E, &w.Einv, &w.Et, &w.rv, &w.ri, &w.z, &w.y, &w.zt, &w.zp, &w.yp, &w.tm2,
                     &w.Ax, &w.zpol, &w.ypol, &w.bb, &w.r2, &w.dd, &w.act, &w.rvp};
    for (double** v : vm) *v = take(m);
    w.L = (n > (size_t)GEN_NMAX) ? take(n * n) : nullptr;
    return w;
}

struct GenResid {
    double prim_res, dual_res, eps_prim, eps_dual;
    double ax_n, z_n, px_n, aty_n, q_n;
    double prim_res_s, dual_res_s;
};

// block-wide max of NV values (each thread's local maxima; all >= 0, NaN ignored like `if (t > a) a = t`)
template <int NV>
__device__ inline void gen_bmax(double (&v)[NV], double* s_red) {
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double x = v[k];
        for (int o = 32; o > 0; o >>= 1) {
            const double y = __shfl_xor(x, o);
            x = (y > x) ? y : x;
        }
        if (lane == 0) s_red[wv * NV + k] = x;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double x = 0.0;
        for (int q = 0; q < GEN_NT / 64; ++q) {
            const double y = s_red[q * NV + k];
            x = (y > x) ? y : x;
        }
        v[k] = x;
    }
    __syncthreads();
}

// y = M x (rows r, cols cdim; mat_vec): one thread per row, sequential dot
__device__ inline void gen_mv(const double* M, int r, int cdim, const double* x, double* y) {
    for (int i = threadIdx.x; i < r; i += GEN_NT) {
        const double* mi = M + (size_t)i * cdim;
        double s = 0.0;
        for (int j = 0; j < cdim; ++j) s += mi[j] * x[j];
        y[i] = s;
    }
}

// y = M' x (mat_tvec): one thread per column, rows in order, zero x entries skipped
__device__ inline void gen_mtv(const double* M, int r, int cdim, const double* x, double* y) {
    for (int j = threadIdx.x; j < cdim; j += GEN_NT) {
        double s = 0.0;
        for (int i = 0; i < r; ++i) {
            const double xi = x[i];
            if (xi == 0.0) continue;
            s += M[(size_t)i * cdim + j] * xi;
        }
        y[j] = s;
    }
}

// K = P + sig I + A' diag(rv) A (lower triangle, factor_kkt's per-entry order) then Cholesky in place
// (lower factor in L[i * LD + j], i >= j; LD = GEN_LD in LDS, n in the caller's scratch).  Returns false if a
// pivot is not positive.
constexpr int GEN_LD = GEN_NMAX + 1;
__device__ inline bool gen_factor(const GenWs& w, const double* rv, int n, int m, double sig, double* L, int LD,
                                  int* s_ok) {
    const int t = threadIdx.x;
    for (int e = t; e < n * n; e += GEN_NT) {
        const int i = e / n, j = e - i * n;
        if (j > i) continue;
        double k = w.P[i * n + j];
        if (i == j) k += sig;
        for (int r = 0; r < m; ++r) {
            const double rr = rv[r];
            if (rr == 0.0) continue;
            const double* a = w.A + (size_t)r * n;
            if (a[i] == 0.0) continue;
            const double tq = rr * a[i];
            k += tq * a[j];
        }
        L[i * LD + j] = k;
    }
    if (t == 0) *s_ok = 1;
    __syncthreads();
    for (int j = 0; j < n; ++j) {
        if (t == 0) {
            const double s = L[j * LD + j];
            if (!(s > 0.0)) *s_ok = 0;
            else L[j * LD + j] = sqrt(s);
        }
        __syncthreads();
        if (!*s_ok) return false;
        const double d = L[j * LD + j];
        for (int i = j + 1 + t; i < n; i += GEN_NT) L[i * LD + j] = L[i * LD + j] / d;
        __syncthreads();
        // trailing update: entry (i, c), i >= c > j, minus L[i][j] L[c][j]
        const int nr = n - j - 1;
        for (int e = t; e < nr * nr; e += GEN_NT) {
            const int ii = e / nr, cc = e - ii * nr;
            if (cc > ii) continue;
            const int i = j + 1 + ii, c = j + 1 + cc;
            L[i * LD + c] -= L[i * LD + j] * L[c * LD + j];
        }
        __syncthreads();
    }
    return true;
}

// b <- K^{-1} b with the factor L (chol_solve): wave 0, lane l owns rows l, l + 64, l + 128, ... (GEN_RMAX)
template <int RMAX>
__device__ inline void gen_solve(const double* L, int LD, int n, double* b) {
    const int t = threadIdx.x;
    if (t < 64) {
        double v[RMAX];
#pragma unroll
        for (int r = 0; r < RMAX; ++r) v[r] = (t + 64 * r < n) ? b[t + 64 * r] : 0.0;
        for (int k = 0; k < n; ++k) {   // forward: row i's terms in ascending k
            const int owner = k & 63, kr = k >> 6;
            double x = 0.0;
#pragma unroll
            for (int r = 0; r < RMAX; ++r) x = (r == kr) ? v[r] : x;
            if (t == owner) x = x / L[k * LD + k];
            const double bk = __shfl(x, owner);
#pragma unroll
            for (int r = 0; r < RMAX; ++r) {
                const int row = t + 64 * r;
                if (r == kr && t == owner) v[r] = bk;
                if (row > k && row < n) v[r] -= L[row * LD + k] * bk;
            }
        }
        for (int k = n - 1; k >= 0; --k) {   // backward: row i's terms in descending k
            const int owner = k & 63, kr = k >> 6;
            double x = 0.0;
#pragma unroll
            for (int r = 0; r < RMAX; ++r) x = (r == kr) ? v[r] : x;
            if (t == owner) x = x / L[k * LD + k];
            const double bk = __shfl(x, owner);
#pragma unroll
            for (int r = 0; r < RMAX; ++r) {
                const int row = t + 64 * r;
                if (r == kr && t == owner) v[r] = bk;
                if (row < k) v[r] -= L[k * LD + row] * bk;
            }
        }
#pragma unroll
        for (int r = 0; r < RMAX; ++r)
            if (t + 64 * r < n) b[t + 64 * r] = v[r];
    }
    __syncthreads();
}

// residuals of (x, z, y) in the unscaled problem (oracle residuals)
__device__ inline void gen_residuals(const GenWs& w, const traj_mpc_config& c, double cinv, int n, int m,
                                     const double* x, const double* z, const double* y, GenResid& r,
                                     double* s_red) {
    const int t = threadIdx.x;
    gen_mv(w.A, m, n, x, w.Ax);
    gen_mv(w.P, n, n, x, w.Px);
    gen_mtv(w.A, m, n, y, w.Aty);
    __syncthreads();
    double v[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    auto mx = [](double& a, double b) { if (b > a) a = b; };
    for (int i = t; i < m; i += GEN_NT) {
        mx(v[0], fabs(w.Einv[i] * (w.Ax[i] - z[i])));
        mx(v[1], fabs(w.Einv[i] * w.Ax[i]));
        mx(v[2], fabs(w.Einv[i] * z[i]));
        mx(v[3], fabs(w.Ax[i] - z[i]));
        mx(v[4], fabs(w.Ax[i]));
        mx(v[5], fabs(z[i]));
    }
    for (int j = t; j < n; j += GEN_NT) {
        const double vv = w.Px[j] + w.q[j] + w.Aty[j];
        mx(v[6], fabs(w.Dinv[j] * vv) * cinv);
        mx(v[7], fabs(w.Dinv[j] * w.Px[j]) * cinv);
        mx(v[8], fabs(w.Dinv[j] * w.Aty[j]) * cinv);
        mx(v[9], fabs(w.Dinv[j] * w.q[j]) * cinv);
        mx(v[10], fabs(vv));
        mx(v[11], fabs(w.Px[j]));
        mx(v[12], fabs(w.Aty[j]));
        mx(v[13], fabs(w.q[j]));
    }
    gen_bmax(v, s_red);
    r.prim_res = v[0];
    r.dual_res = v[6];
    r.eps_prim = c.eps_abs + c.eps_rel * (v[1] > v[2] ? v[1] : v[2]);
    double m2 = v[7] > v[8] ? v[7] : v[8];
    if (v[9] > m2) m2 = v[9];
    r.eps_dual = c.eps_abs + c.eps_rel * m2;
    r.prim_res_s = v[3];
    r.dual_res_s = v[10];
    r.ax_n = v[4];
    r.z_n = v[5];
    r.px_n = v[11];
    r.aty_n = v[12];
    r.q_n = v[13];
}

// OSQP is_primal_infeasible on dy = y - y_prev (oracle primal_infeasible)
__device__ inline bool gen_prim_inf(const GenWs& w, const traj_mpc_config& c, int n, int m, double* s_red,
                                    double* s_v) {
    const int t = threadIdx.x;
    double v[1] = {0.0};
    for (int i = t; i < m; i += GEN_NT) {
        double d = w.y[i] - w.yp[i];
        if (w.u[i] >= INFTY * MIN_SCALING && d > 0.0) d = 0.0;
        if (w.l[i] <= -INFTY * MIN_SCALING && d < 0.0) d = 0.0;
        w.dd[i] = d;
        const double a = fabs(w.E[i] * d);
        if (a > v[0]) v[0] = a;
    }
    gen_bmax(v, s_red);   // (syncs: dd visible)
    const double nrm = v[0];
    if (!(nrm > DIV_TOL)) return false;
    if (t == 0) {
        double lhs = 0.0;
        for (int i = 0; i < m; ++i) {
            const double d = w.dd[i];
            if (d > 0.0) lhs += w.u[i] * d;
            else if (d < 0.0) lhs += w.l[i] * d;
        }
        s_v[0] = lhs;
    }
    __syncthreads();
    const double lhs = s_v[0];
    __syncthreads();
    if (!(lhs < -c.eps_prim_inf * nrm)) return false;
    gen_mtv(w.A, m, n, w.dd, w.tt);
    __syncthreads();
    double an[1] = {0.0};
    for (int j = t; j < n; j += GEN_NT) {
        const double a = fabs(w.Dinv[j] * w.tt[j]);
        if (a > an[0]) an[0] = a;
    }
    gen_bmax(an, s_red);
    return an[0] < c.eps_prim_inf * nrm;
}

// active set of (z, y) (OSQP form_Ared): -1 lower, +1 upper, 0 inactive
__device__ inline void gen_active(const GenWs& w, int m, const double* z, const double* y) {
    for (int i = threadIdx.x; i < m; i += GEN_NT) {
        double a = 0.0;
        if (z[i] - w.l[i] < -y[i]) a = -1.0;
        else if (w.u[i] - z[i] < y[i]) a = 1.0;
        w.act[i] = a;
    }
    __syncthreads();
}

// reduced-KKT solve for the active set w.act (kkt_solve_active): x -> w.xpol, y -> w.ypol, A x -> w.Ax
template <int RMAX>
__device__ inline bool gen_kkt_active(const GenWs& w, const traj_mpc_config& c, int n, int m, double* L, int LD,
                                      int* s_ok) {
    const int t = threadIdx.x;
    const double dlt = c.delta;
    for (int i = t; i < m; i += GEN_NT) {
        const double a = w.act[i];
        w.bb[i] = a < 0.0 ? w.l[i] : (a > 0.0 ? w.u[i] : 0.0);
        w.rvp[i] = (a != 0.0) ? 1.0 / dlt : 0.0;
    }
    __syncthreads();
    if (!gen_factor(w, w.rvp, n, m, dlt, L, LD, s_ok)) return false;
    for (int j = t; j < n; j += GEN_NT) {
        w.xpol[j] = 0.0;
        w.r1[j] = -w.q[j];
    }
    for (int i = t; i < m; i += GEN_NT) {
        w.ypol[i] = 0.0;
        w.r2[i] = (w.act[i] != 0.0) ? w.bb[i] : 0.0;
    }
    __syncthreads();
    for (int pass = 0; pass <= c.polish_refine_iter; ++pass) {
        for (int j = t; j < n; j += GEN_NT) {
            double s = w.r1[j];
            for (int i = 0; i < m; ++i) {
                if (w.act[i] == 0.0) continue;
                const double sc = w.r2[i] / dlt;
                s += w.A[(size_t)i * n + j] * sc;
            }
            w.tt[j] = s;
        }
        __syncthreads();
        gen_solve<RMAX>(L, LD, n, w.tt);
        gen_mv(w.A, m, n, w.tt, w.Ax);
        __syncthreads();
        for (int j = t; j < n; j += GEN_NT) w.xpol[j] += w.tt[j];
        for (int i = t; i < m; i += GEN_NT)
            if (w.act[i] != 0.0) w.ypol[i] += (w.Ax[i] - w.r2[i]) / dlt;
        __syncthreads();
        if (pass == c.polish_refine_iter) break;
        gen_mv(w.P, n, n, w.xpol, w.r1);
        gen_mtv(w.A, m, n, w.ypol, w.tt);
        __syncthreads();
        for (int j = t; j < n; j += GEN_NT) w.r1[j] = -w.q[j] - w.r1[j] - w.tt[j];
        gen_mv(w.A, m, n, w.xpol, w.Ax);
        __syncthreads();
        for (int i = t; i < m; i += GEN_NT) w.r2[i] = (w.act[i] != 0.0) ? w.bb[i] - w.Ax[i] : 0.0;
        __syncthreads();
    }
    gen_mv(w.A, m, n, w.xpol, w.Ax);
    __syncthreads();
    return true;
}

template <int RMAX>
__global__ __launch_bounds__(GEN_NT) void solve_gen_kernel(const KArgs a, double* gws, size_t gstride) {
    __shared__ double s_L[GEN_NMAX * GEN_LD];
    __shared__ double s_red[4 * 14];
    __shared__ double s_v[8];
    __shared__ int s_i[8];
    const int b = blockIdx.x, t = threadIdx.x;
    const traj_mpc_config& c = a.c;
    const int N = c.N, n = 2 * N;
    const GenWs w = gen_carve(gws + (size_t)b * gstride, N);
    // the factor: LDS up to the hot kernels' capacity, the caller's scratch past it
    double* const s_Lf = (n <= GEN_NMAX) ? s_L : w.L;
    const int LD = (n <= GEN_NMAX) ? GEN_LD : n;
    const double* x0 = a.x0 + 6 * (size_t)b;
    const double* up = a.u_prev + 2 * (size_t)b;
    const double* pref = a.path_ref + (size_t)3 * (N + 1) * b;
    const double* vr = a.vref + (size_t)(N + 1) * b;
    const double* Adk = a.Ad + (size_t)36 * N * b;
    const double* Bdk = a.Bd + (size_t)12 * N * b;
    const double* gdk = a.gd + (size_t)6 * N * b;

    // state rows (count_state_rows): one per state with a finite side, for k = 1..N
    int nsr = 0;
    for (int i = 0; i < 6; ++i) {
        const double lo = c.has_x_lo ? c.x_lo[i] : -INFINITY, hi = c.has_x_hi ? c.x_hi[i] : INFINITY;
        if (lo > -INFTY || hi < INFTY) ++nsr;
    }
    const int m = 4 * N + nsr * N;

    int status = TRAJ_STATUS_SOLVER_ERROR, iter = 0, pol = 0;
    // ---- inputs finite (orc_mpc_step_warm) ----
    if (t == 0) {
        int ok = 1;
        for (int i = 0; i < 6; ++i) ok &= isfinite(x0[i]) ? 1 : 0;
        for (int i = 0; i < 2; ++i) ok &= isfinite(up[i]) ? 1 : 0;
        for (int i = 0; i < 3 * (N + 1); ++i) ok &= isfinite(pref[i]) ? 1 : 0;
        for (int i = 0; i <= N; ++i) ok &= isfinite(vr[i]) ? 1 : 0;
        s_i[0] = ok;
    }
    __syncthreads();
    const bool inputs_ok = s_i[0] != 0;
    __syncthreads();

    if (inputs_ok) {
        // ---- build_qp: free response xh and sensitivities G[k] (6 x n) ----
        for (int e = t; e < 6 * (N + 1) * n; e += GEN_NT) w.G[e] = 0.0;
        if (t < 6) w.xh[t] = x0[t];
        __syncthreads();
        for (int k = 0; k < N; ++k) {
            const double* A = Adk + 36 * k;
            const double* Bm = Bdk + 12 * k;
            if (t < 6) {
                double s = 0.0;
                for (int cc = 0; cc < 6; ++cc) s += A[t * 6 + cc] * w.xh[k * 6 + cc];
                w.xh[(k + 1) * 6 + t] = s + gdk[6 * k + t];
            }
            const double* Gk = w.G + (size_t)k * 6 * n;
            double* Gk1 = w.G + (size_t)(k + 1) * 6 * n;
            for (int e = t; e < 6 * (2 * k + 2); e += GEN_NT) {
                const int r = e / (2 * k + 2), j = e - r * (2 * k + 2);
                if (j < 2 * k) {
                    double s = 0.0;
                    for (int cc = 0; cc < 6; ++cc) s += A[r * 6 + cc] * Gk[cc * n + j];
                    Gk1[r * n + j] = s;
                } else {
                    Gk1[r * n + j] = Bm[r * 2 + (j - 2 * k)];
                }
            }
            __syncthreads();
        }
        // ---- tracking cost (:217-228, :243-247) ----
        for (int e = t; e < n * n; e += GEN_NT) w.P[e] = 0.0;
        for (int j = t; j < n; j += GEN_NT) w.q[j] = 0.0;
        __syncthreads();
        const double W[3] = {c.q_c, c.q_phi, c.q_vx};
        double cst = 0.0;   // thread 0's copy is the one used
        for (int k = 0; k <= N; ++k) {
            const double Xr = pref[k * 3 + 0], Yr = pref[k * 3 + 1], Pr = pref[k * 3 + 2];
            double s, co;
            pm_sincos(Pr, &s, &co);
            const double* xk = w.xh + 6 * k;
            double e3[3];
            e3[0] = s * (xk[0] - Xr) - co * (xk[1] - Yr);
            e3[1] = xk[2] - Pr;
            e3[2] = xk[3] - vr[k];
            for (int q3 = 0; q3 < 3; ++q3) cst += W[q3] * e3[q3] * e3[q3];
            if (k == 0) continue;
            const double* Gk = w.G + (size_t)k * 6 * n;
            for (int j = t; j < n; j += GEN_NT) {
                w.F[0 * n + j] = s * Gk[0 * n + j] - co * Gk[1 * n + j];
                w.F[1 * n + j] = Gk[2 * n + j];
                w.F[2 * n + j] = Gk[3 * n + j];
            }
            __syncthreads();
            const int nk = 2 * k;
            for (int e = t; e < nk * nk; e += GEN_NT) {
                const int i = e / nk, j = e - i * nk;
                double pv = w.P[i * n + j];
                for (int q3 = 0; q3 < 3; ++q3) {
                    const double wi = 2.0 * W[q3] * w.F[q3 * n + i];
                    pv += wi * w.F[q3 * n + j];
                }
                w.P[i * n + j] = pv;
            }
            for (int i = t; i < nk; i += GEN_NT) {
                double qv = w.q[i];
                for (int q3 = 0; q3 < 3; ++q3) {
                    const double wi = 2.0 * W[q3] * w.F[q3 * n + i];
                    qv += wi * e3[q3];
                }
                w.q[i] = qv;
            }
            __syncthreads();
        }
        // ---- input cost U'RU + dU'Rd dU (:230-240), serial like the oracle ----
        if (t == 0) {
            double Rs[4], Rds[4];
            Rs[0] = c.R[0]; Rs[3] = c.R[3]; Rs[1] = Rs[2] = 0.5 * (c.R[1] + c.R[2]);
            Rds[0] = c.Rd[0]; Rds[3] = c.Rd[3]; Rds[1] = Rds[2] = 0.5 * (c.Rd[1] + c.Rd[2]);
            for (int k = 0; k < N; ++k)
                for (int aa = 0; aa < 2; ++aa)
                    for (int bb = 0; bb < 2; ++bb) {
                        w.P[(2 * k + aa) * n + 2 * k + bb] += 2.0 * Rs[aa * 2 + bb];
                        w.P[(2 * k + aa) * n + 2 * k + bb] += 2.0 * Rds[aa * 2 + bb];
                        if (k > 0) {
                            w.P[(2 * k - 2 + aa) * n + 2 * k - 2 + bb] += 2.0 * Rds[aa * 2 + bb];
                            w.P[(2 * k + aa) * n + 2 * k - 2 + bb] -= 2.0 * Rds[aa * 2 + bb];
                            w.P[(2 * k - 2 + aa) * n + 2 * k + bb] -= 2.0 * Rds[aa * 2 + bb];
                        }
                    }
            for (int aa = 0; aa < 2; ++aa) {
                double tq = 0.0;
                for (int bb = 0; bb < 2; ++bb) tq += Rds[aa * 2 + bb] * up[bb];
                w.q[aa] -= 2.0 * tq;
                cst += up[aa] * tq;
            }
        }
        // ---- constraint rows (:195-213): stage-major box/rate rows, then the state rows ----
        for (int e = t; e < m * n; e += GEN_NT) w.A[e] = 0.0;
        __syncthreads();
        for (int e = t; e < 2 * N; e += GEN_NT) {
            const int k = e >> 1, ch = e & 1;
            const int rb = 4 * k + ch, rr = 4 * k + 2 + ch, j = 2 * k + ch;
            w.A[(size_t)rb * n + j] = 1.0;
            w.l[rb] = c.u_lo[ch];
            w.u[rb] = c.u_hi[ch];
            w.A[(size_t)rr * n + j] = 1.0;
            if (k > 0) {
                w.A[(size_t)rr * n + j - 2] = -1.0;
                w.l[rr] = c.du_lo[ch];
                w.u[rr] = c.du_hi[ch];
            } else {
                w.l[rr] = c.du_lo[ch] + up[ch];
                w.u[rr] = c.du_hi[ch] + up[ch];
            }
        }
        int infeasible_const = 0;
        {
            int row = 4 * N;
            for (int i = 0; i < 6; ++i) {
                const double lo = c.has_x_lo ? c.x_lo[i] : -INFINITY, hi = c.has_x_hi ? c.x_hi[i] : INFINITY;
                if (!(lo > -INFTY || hi < INFTY)) continue;
                if (x0[i] < lo || x0[i] > hi) infeasible_const = 1;   // k = 0: X_0 == x0
                for (int k = 1; k <= N; ++k, ++row) {
                    const double* Gk = w.G + (size_t)k * 6 * n;
                    for (int j = t; j < n; j += GEN_NT) w.A[(size_t)row * n + j] = Gk[i * n + j];
                    if (t == 0) {
                        w.l[row] = (lo > -INFTY) ? lo - w.xh[6 * k + i] : -INFINITY;
                        w.u[row] = (hi < INFTY) ? hi - w.xh[6 * k + i] : INFINITY;
                    }
                }
            }
        }
        __syncthreads();
        // ---- finite data, constant infeasibility, box/rate chain feasibility ----
        {
            int bad = 0;
            for (int e = t; e < n * n; e += GEN_NT) bad |= !isfinite(w.P[e]);
            for (int e = t; e < n; e += GEN_NT) bad |= !isfinite(w.q[e]);
            for (int e = t; e < m * n; e += GEN_NT) bad |= !isfinite(w.A[e]);
            if (t == 0) s_i[1] = 0;
            __syncthreads();
            if (bad) s_i[1] = 1;
            if (t == 0) {
                int feas = 1;
                for (int ch = 0; ch < 2; ++ch) {
                    double lo = up[ch], hi = up[ch];
                    for (int k = 0; k < N; ++k) {
                        double nlo = lo + c.du_lo[ch], nhi = hi + c.du_hi[ch];
                        if (nlo < c.u_lo[ch]) nlo = c.u_lo[ch];
                        if (nhi > c.u_hi[ch]) nhi = c.u_hi[ch];
                        if (!(nlo <= nhi)) feas = 0;
                        lo = nlo;
                        hi = nhi;
                    }
                }
                s_i[2] = feas;
                s_v[0] = cst;
            }
            __syncthreads();
        }
        const bool data_ok = s_i[1] == 0, feasible = !infeasible_const && s_i[2] != 0;
        __syncthreads();
        if (!data_ok) status = TRAJ_STATUS_SOLVER_ERROR;
        else if (!feasible) status = TRAJ_STATUS_INFEASIBLE;
        else {
            // ---- osqp_solve ----
            double rho = c.rho, cc = 1.0, cinv = 1.0;
            for (int j = t; j < n; j += GEN_NT) w.D[j] = 1.0;
            for (int i = t; i < m; i += GEN_NT) w.E[i] = 1.0;
            __syncthreads();
            for (int it = 0; it < c.scaling_iters; ++it) {   // osqp_scale
                for (int j = t; j < n; j += GEN_NT) {
                    double am = 0.0;
                    for (int i = 0; i < n; ++i) { const double v = fabs(w.P[i * n + j]); if (v > am) am = v; }
                    for (int i = 0; i < m; ++i) { const double v = fabs(w.A[(size_t)i * n + j]); if (v > am) am = v; }
                    w.Dt[j] = 1.0 / sqrt(limit_scaling(am));
                }
                for (int i = t; i < m; i += GEN_NT) {
                    double am = 0.0;
                    for (int j = 0; j < n; ++j) { const double v = fabs(w.A[(size_t)i * n + j]); if (v > am) am = v; }
                    w.Et[i] = 1.0 / sqrt(limit_scaling(am));
                }
                __syncthreads();
                for (int e = t; e < n * n; e += GEN_NT) {
                    const int i = e / n, j = e - i * n;
                    w.P[e] *= w.Dt[i] * w.Dt[j];
                }
                for (int e = t; e < m * n; e += GEN_NT) {
                    const int i = e / n, j = e - i * n;
                    w.A[e] *= w.Et[i] * w.Dt[j];
                }
                for (int j = t; j < n; j += GEN_NT) { w.q[j] *= w.Dt[j]; w.D[j] *= w.Dt[j]; }
                for (int i = t; i < m; i += GEN_NT) w.E[i] *= w.Et[i];
                __syncthreads();
                // cost scaling: mean of the column maxima (sequential sum), |q|_inf
                for (int j = t; j < n; j += GEN_NT) {
                    double am = 0.0;
                    for (int i = 0; i < n; ++i) { const double v = fabs(w.P[i * n + j]); if (v > am) am = v; }
                    w.tt[j] = am;
                }
                double qn[1] = {0.0};
                for (int j = t; j < n; j += GEN_NT) { const double v = fabs(w.q[j]); if (v > qn[0]) qn[0] = v; }
                gen_bmax(qn, s_red);
                if (t == 0) {
                    double mean = 0.0;
                    for (int j = 0; j < n; ++j) mean += w.tt[j];
                    mean /= n;
                    const double ql = limit_scaling(qn[0]);
                    double ct = mean > ql ? mean : ql;
                    ct = 1.0 / limit_scaling(ct);
                    s_v[1] = ct;
                }
                __syncthreads();
                const double ct = s_v[1];
                for (int e = t; e < n * n; e += GEN_NT) w.P[e] *= ct;
                for (int j = t; j < n; j += GEN_NT) w.q[j] *= ct;
                cc *= ct;
                __syncthreads();
            }
            for (int j = t; j < n; j += GEN_NT) w.Dinv[j] = 1.0 / w.D[j];
            for (int i = t; i < m; i += GEN_NT) {
                w.Einv[i] = 1.0 / w.E[i];
                if (w.l[i] > -INFTY) w.l[i] *= w.E[i]; else w.l[i] = -INFTY;
                if (w.u[i] < INFTY) w.u[i] *= w.E[i]; else w.u[i] = INFTY;
            }
            cinv = 1.0 / cc;
            auto set_rho = [&]() {
                for (int i = t; i < m; i += GEN_NT) {
                    double r;
                    if (w.l[i] <= -INFTY * MIN_SCALING && w.u[i] >= INFTY * MIN_SCALING) r = RHO_MIN;
                    else if (w.u[i] - w.l[i] < RHO_TOL) r = RHO_EQ_OVER_INEQ * rho;
                    else r = rho;
                    w.rv[i] = r;
                    w.ri[i] = 1.0 / r;
                }
                __syncthreads();
            };
            for (int j = t; j < n; j += GEN_NT) w.x[j] = 0.0;
            for (int i = t; i < m; i += GEN_NT) { w.z[i] = 0.0; w.y[i] = 0.0; }
            __syncthreads();
            set_rho();
            if (gen_factor(w, w.rv, n, m, c.sigma, s_Lf, LD, &s_i[3])) {
                GenResid r = {};
                int converged = 0, rounds = 0;
                bool infeasible = false, fail = false;
                double escale = 1.0;
                iter = 1;
                for (;;) {   // ADMM (+ exact-mode continuation rounds)
                    for (; iter <= c.max_iter; ++iter) {
                        for (int j = t; j < n; j += GEN_NT) w.xp[j] = w.x[j];
                        for (int i = t; i < m; i += GEN_NT) {
                            w.zp[i] = w.z[i];
                            w.yp[i] = w.y[i];
                            w.tm2[i] = w.rv[i] * w.z[i] - w.y[i];
                        }
                        __syncthreads();
                        gen_mtv(w.A, m, n, w.tm2, w.rhs);
                        __syncthreads();
                        for (int j = t; j < n; j += GEN_NT) w.xt[j] = w.rhs[j] + (c.sigma * w.xp[j] - w.q[j]);
                        __syncthreads();
                        gen_solve<RMAX>(s_Lf, LD, n, w.xt);
                        gen_mv(w.A, m, n, w.xt, w.zt);
                        __syncthreads();
                        for (int j = t; j < n; j += GEN_NT) w.x[j] = c.alpha * w.xt[j] + (1.0 - c.alpha) * w.xp[j];
                        for (int i = t; i < m; i += GEN_NT) {
                            const double zr = c.alpha * w.zt[i] + (1.0 - c.alpha) * w.zp[i];
                            const double v = zr + w.ri[i] * w.y[i];
                            const double zz = v < w.l[i] ? w.l[i] : (v > w.u[i] ? w.u[i] : v);
                            w.z[i] = zz;
                            w.y[i] = w.y[i] + w.rv[i] * (zr - zz);
                        }
                        __syncthreads();
                        if (iter % c.check_interval == 0) {
                            gen_residuals(w, c, cinv, n, m, w.x, w.z, w.y, r, s_red);
                            if (r.prim_res <= escale * r.eps_prim && r.dual_res <= escale * r.eps_dual) {
                                converged = 1;
                                break;
                            }
                            if (gen_prim_inf(w, c, n, m, s_red, s_v)) { infeasible = true; break; }
                            if (c.adaptive_rho) {
                                const double pn = r.ax_n > r.z_n ? r.ax_n : r.z_n;
                                double dn = r.px_n > r.aty_n ? r.px_n : r.aty_n;
                                if (r.q_n > dn) dn = r.q_n;
                                const double prr = r.prim_res_s / (pn + DIV_TOL);
                                const double drr = r.dual_res_s / (dn + DIV_TOL);
                                double est = rho * sqrt(prr / (drr + DIV_TOL));
                                if (est < RHO_MIN) est = RHO_MIN;
                                if (est > RHO_MAX) est = RHO_MAX;
                                if (est > rho * c.adaptive_rho_tol || est < rho / c.adaptive_rho_tol) {
                                    rho = est;
                                    set_rho();
                                    if (!gen_factor(w, w.rv, n, m, c.sigma, s_Lf, LD, &s_i[3])) { fail = true; break; }
                                }
                            }
                        }
                    }
                    if (infeasible) { status = TRAJ_STATUS_INFEASIBLE; break; }
                    if (fail) { status = TRAJ_STATUS_SOLVER_ERROR; break; }
                    if (converged) status = TRAJ_STATUS_OPTIMAL;
                    else {
                        iter = c.max_iter;
                        gen_residuals(w, c, cinv, n, m, w.x, w.z, w.y, r, s_red);
                        if (rounds > 0 && r.prim_res <= r.eps_prim && r.dual_res <= r.eps_dual)
                            status = TRAJ_STATUS_OPTIMAL;
                        else if (r.prim_res <= 10.0 * r.eps_prim && r.dual_res <= 10.0 * r.eps_dual)
                            status = TRAJ_STATUS_OPTIMAL_INACCURATE;
                        else status = TRAJ_STATUS_USER_LIMIT;
                    }
                    pol = 0;
                    if (status == TRAJ_STATUS_OPTIMAL && c.polish && c.polish_mode == 1) {
                        // exact_polish: reduced solves as a primal-dual active-set method, KKT-certified
                        gen_active(w, m, w.z, w.y);
                        int cert = 0, pass;
                        const double tol = c.cert_tol;
                        for (pass = 1; pass <= c.polish_max_pass; ++pass) {
                            if (!gen_kkt_active<RMAX>(w, c, n, m, s_Lf, LD, &s_i[3])) break;
                            gen_mv(w.P, n, n, w.xpol, w.Px);
                            gen_mtv(w.A, m, n, w.ypol, w.Aty);
                            __syncthreads();
                            double v[2] = {0.0, 1.0};
                            for (int j = t; j < n; j += GEN_NT) {
                                const double st = fabs(w.Dinv[j] * (w.Px[j] + w.q[j] + w.Aty[j])) * cinv;
                                if (st > v[0]) v[0] = st;
                                double s1 = fabs(w.Dinv[j] * w.q[j]) * cinv; if (s1 > v[1]) v[1] = s1;
                                s1 = fabs(w.Dinv[j] * w.Px[j]) * cinv; if (s1 > v[1]) v[1] = s1;
                            }
                            gen_bmax(v, s_red);
                            const double gsc = v[1];
                            double badv[1] = {v[0] <= tol * gsc ? 0.0 : 1.0};
                            for (int i = t; i < m; i += GEN_NT) {
                                const double ax = w.Ax[i] * w.Einv[i];
                                if (w.l[i] > -INFTY) { const double lo = w.l[i] * w.Einv[i]; if (ax < lo - tol * (1.0 + fabs(lo))) badv[0] = 1.0; }
                                if (w.u[i] < INFTY) { const double hi = w.u[i] * w.Einv[i]; if (ax > hi + tol * (1.0 + fabs(hi))) badv[0] = 1.0; }
                                const double yu = w.ypol[i] * w.E[i] * cinv;
                                if (w.act[i] < 0.0 && yu > tol * gsc) badv[0] = 1.0;
                                if (w.act[i] > 0.0 && yu < -tol * gsc) badv[0] = 1.0;
                            }
                            gen_bmax(badv, s_red);
                            if (badv[0] == 0.0) { cert = 1; break; }
                            gen_active(w, m, w.Ax, w.ypol);
                        }
                        if (cert) {
                            for (int j = t; j < n; j += GEN_NT) w.x[j] = w.xpol[j];
                            for (int i = t; i < m; i += GEN_NT) {
                                const double ax = w.Ax[i];
                                w.z[i] = ax < w.l[i] ? w.l[i] : (ax > w.u[i] ? w.u[i] : ax);
                                w.y[i] = w.ypol[i];
                            }
                            __syncthreads();
                            gen_residuals(w, c, cinv, n, m, w.x, w.z, w.y, r, s_red);
                            pol = pass + 16 * rounds;
                        }
                        if (!pol && rounds < c.polish_max_rounds && iter < c.max_iter) {
                            // not certified: continue ADMM to a 100x tighter tolerance and polish again
                            ++rounds;
                            escale *= 1e-2;
                            converged = 0;
                            ++iter;
                            set_rho();   // the ADMM factor (the polish overwrote it): same rho, same bits
                            if (!gen_factor(w, w.rv, n, m, c.sigma, s_Lf, LD, &s_i[3])) {
                                status = TRAJ_STATUS_SOLVER_ERROR;
                                break;
                            }
                            continue;
                        }
                    } else if (status == TRAJ_STATUS_OPTIMAL && c.polish) {
                        // osqp_polish + OSQP's acceptance rule
                        gen_active(w, m, w.z, w.y);
                        if (gen_kkt_active<RMAX>(w, c, n, m, s_Lf, LD, &s_i[3])) {
                            for (int i = t; i < m; i += GEN_NT) {
                                const double ztv = w.Ax[i] + w.ypol[i];
                                const double zz = ztv < w.l[i] ? w.l[i] : (ztv > w.u[i] ? w.u[i] : ztv);
                                w.zpol[i] = zz;
                                w.dd[i] = ztv - zz;   // polished y
                            }
                            __syncthreads();
                            GenResid rp = {};
                            gen_residuals(w, c, cinv, n, m, w.xpol, w.zpol, w.dd, rp, s_red);
                            const bool ok = (rp.prim_res < r.prim_res && rp.dual_res < r.dual_res) ||
                                            (rp.prim_res < r.prim_res && r.dual_res < 1e-10) ||
                                            (rp.dual_res < r.dual_res && r.prim_res < 1e-10);
                            if (ok) {
                                for (int j = t; j < n; j += GEN_NT) w.x[j] = w.xpol[j];
                                for (int i = t; i < m; i += GEN_NT) { w.z[i] = w.zpol[i]; w.y[i] = w.dd[i]; }
                                __syncthreads();
                                r = rp;
                                pol = 1;
                            }
                        }
                    }
                    break;
                }
                if (iter > c.max_iter) iter = c.max_iter;
                for (int j = t; j < n; j += GEN_NT) w.xs[j] = w.D[j] * w.x[j];
                __syncthreads();
            } else {
                status = TRAJ_STATUS_SOLVER_ERROR;   // factorization failed before the first iteration
                iter = 0;
            }
        }
    }
    __syncthreads();

    // ---- outputs (orc_mpc_step_warm): U, X by the linear model, objective, u_cmd ----
    const bool good = inputs_ok && (status == TRAJ_STATUS_OPTIMAL || status == TRAJ_STATUS_OPTIMAL_INACCURATE);
    const double nan = __builtin_nan("");
    double* U = w.U;
    double* X = w.G;   // G is no longer needed: X [6][N+1]
    if (good) {
        for (int k = t; k < N; k += GEN_NT) { U[k] = w.xs[2 * k]; U[N + k] = w.xs[2 * k + 1]; }
        if (t < 6) X[t * (N + 1)] = x0[t];
        __syncthreads();
        if (t < 6) {
            for (int k = 0; k < N; ++k) {
                const double* A = Adk + 36 * k;
                const double* Bm = Bdk + 12 * k;
                const double* g = gdk + 6 * k;
                double s = 0.0;
                for (int cc = 0; cc < 6; ++cc) s += A[t * 6 + cc] * X[cc * (N + 1) + k];
                s += Bm[t * 2] * U[k] + Bm[t * 2 + 1] * U[N + k] + g[t];
                X[t * (N + 1) + k + 1] = s;
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        double obj = nan;
        if (good) {
            obj = 0.0;
            for (int k = 0; k <= N; ++k) {
                const double ec = lateral_error(X[0 * (N + 1) + k], X[1 * (N + 1) + k], pref[3 * k], pref[3 * k + 1],
                                                pref[3 * k + 2]);
                const double ep = X[2 * (N + 1) + k] - pref[3 * k + 2];
                const double ev = X[3 * (N + 1) + k] - vr[k];
                obj += c.q_c * ec * ec + c.q_phi * ep * ep + c.q_vx * ev * ev;
                if (k == N) break;
                const double uk[2] = {U[k], U[N + k]};
                double du[2];
                for (int aa = 0; aa < 2; ++aa) du[aa] = uk[aa] - (k == 0 ? up[aa] : U[aa * N + k - 1]);
                for (int aa = 0; aa < 2; ++aa)
                    for (int bb = 0; bb < 2; ++bb)
                        obj += uk[aa] * c.R[aa * 2 + bb] * uk[bb] + du[aa] * c.Rd[aa * 2 + bb] * du[bb];
            }
        }
        a.u_cmd[2 * b] = good ? U[0] : up[0];
        a.u_cmd[2 * b + 1] = good ? U[N] : up[1];
        a.status[b] = status;
        if (a.objective) a.objective[b] = obj;
        if (a.iters) a.iters[b] = iter;
        if (a.polished) a.polished[b] = pol;
    }
    if (a.U_opt)
        for (int e = t; e < 2 * N; e += GEN_NT) a.U_opt[(size_t)b * 2 * N + e] = good ? U[e] : nan;
    if (a.X_opt)
        for (int e = t; e < 6 * (N + 1); e += GEN_NT) a.X_opt[(size_t)b * 6 * (N + 1) + e] = good ? X[e] : nan;
}

}  // namespace tgmpc
