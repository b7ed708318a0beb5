/*
 * traj_oracle.c -- CPU ORACLE (test infrastructure only; see traj_oracle.h).
 *
 * Every function cites the reference lines it restates.  Arithmetic order in
 * the physics follows the reference's numpy expressions term by term and the
 * file is compiled with -ffp-contract=off so no FMA contraction reorders it;
 * transcendental results can still differ from numpy's in the last ulp
 * (numpy ships its own SIMD libm), so parity with the reference is stated as a
 * tolerance, never as bit-equality (DESIGN.md "Parity").
 */
#include "traj_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_INFTY 1e30
#define ORC_DIV_TOL 1e-30
#define ORC_MIN_SCALING 1e-4
#define ORC_MAX_SCALING 1e4
#define ORC_RHO_MIN 1e-6
#define ORC_RHO_MAX 1e6
#define ORC_RHO_TOL 1e-4
#define ORC_RHO_EQ_OVER_INEQ 1e3

/* ------------------------------------------------------------------ params */

/* MPC/mpc_6stati.py:9-19 */
void orc_default_params(orc_params* p) {
    p->Cm1 = 0.287; p->Cm2 = 0.0545; p->Cr0 = 0.0518; p->Cr2 = 0.00035;
    p->Br = 3.3852; p->Cr = 1.2691; p->Dr = 0.1737;
    p->Bf = 2.579; p->Cf = 1.2; p->Df = 0.192;
    p->m = 0.041; p->Iz = 27.8e-6; p->lf = 0.029; p->lr = 0.033;
    p->g = 9.81; p->maxAlpha = 0.6; p->vx_zero = 0.3;
}

/* mpc_step kwargs mpc_6stati.py:120-143 + CVXPY's OSQP defaults */
void orc_default_cfg(orc_mpc_cfg* c, int N, double Ts) {
    memset(c, 0, sizeof(*c));
    c->N = N; c->Ts = Ts;
    c->q_c = 6.0; c->q_phi = 0.5; c->q_vx = 0.5;
    c->R[0] = 0.02; c->R[3] = 2.0;
    c->Rd[0] = 0.01; c->Rd[3] = 5.0;
    c->u_lo[0] = -1.0; c->u_hi[0] = 1.0; c->u_lo[1] = -0.6; c->u_hi[1] = 0.6;
    c->du_lo[0] = -0.5; c->du_hi[0] = 0.5; c->du_lo[1] = -0.3; c->du_hi[1] = 0.3;
    c->eps_abs = 1e-5; c->eps_rel = 1e-5; c->eps_prim_inf = 1e-4;
    c->rho = 0.1; c->sigma = 1e-6; c->alpha = 1.6; c->delta = 1e-6;
    c->max_iter = 10000; c->check_interval = 25; c->scaling_iters = 10;
    c->polish = 1; c->polish_refine_iter = 3; c->adaptive_rho = 1; c->adaptive_rho_tol = 5.0;
    c->polish_mode = 0; c->polish_max_pass = 8; c->cert_tol = 1e-9; c->polish_max_rounds = 2;
    c->warm_start = 0;
    c->solver = 1; c->ipm_max_iter = 50; c->ipm_tol = 1e-10;
}

/* ----------------------------------------------------------------- physics */

/* mpc_6stati.py:21-23: np.minimum(np.maximum(x, lo), hi) (NaN propagates) */
double orc_clamp(double x, double lo, double hi) {
    double t = (x < lo) ? lo : x;
    return (t > hi) ? hi : t;
}

/* np.sign: +1 / -1 / 0 (+0.0 for both zeros) / NaN */
static double np_sign(double x) {
    if (x > 0.0) return 1.0;
    if (x < 0.0) return -1.0;
    if (x == 0.0) return 0.0;
    return x;
}

/* The tire sine sin(C atan(B alpha)) (mpc_6stati.py:46-47).  Mode 0 (default): libm's sin, what the reference
 * fixtures pin.  Mode 1: the GPU's bounded-range polynomial, restated coefficient for coefficient and in the same
 * Horner/fma order as trajmpc's physics.h tire_sin_poly (odd Taylor polynomial through x^21 on |z| <= pi/2, libm's
 * sin outside), so that the oracle and the HIP path evaluate the same tire physics and a parity gate that compares
 * unconverged points (the 10,000-iteration cap) tests the solver, not the sine.  Process-global; set it before a
 * batch runs (orc_set_tire_sine). */
static int g_tire_sine = 0;
int orc_set_tire_sine(int mode) {
    int prev = g_tire_sine;
    g_tire_sine = mode ? 1 : 0;
    return prev;
}
static double tire_sin_poly(double x) {
    const double x2 = x * x;
    double q = 1.9572941063391263e-20;
    q = fma(q, x2, -8.22063524662433e-18);
    q = fma(q, x2, 2.8114572543455206e-15);
    q = fma(q, x2, -7.647163731819816e-13);
    q = fma(q, x2, 1.6059043836821613e-10);
    q = fma(q, x2, -2.505210838544172e-08);
    q = fma(q, x2, 2.7557319223985893e-06);
    q = fma(q, x2, -0.0001984126984126984);
    q = fma(q, x2, 0.008333333333333333);
    q = fma(q, x2, -0.16666666666666666);
    return fma(x2 * x, q, x);
}
static double tire_sin(double z) {
    if (g_tire_sine && fabs(z) <= 1.5707963267948966) return tire_sin_poly(z);
    return sin(z);
}
double orc_tire_sin(double z) { return tire_sin(z); }

/* mpc_6stati.py:25-53 */
void orc_tire_forces(const orc_params* p, const double x[6], const double u[2], double out[3]) {
    double vx = x[3], vy = x[4], omega = x[5];
    double d = u[0], delta = u[1];
    double avx = fabs(vx);
    double mx = (p->vx_zero > avx) ? p->vx_zero : avx;       /* python max(abs(vx), vx_zero) */
    double vx_eff = np_sign(vx) * mx;
    double alpha_f = -atan2(omega * p->lf + vy, vx_eff) + delta;
    double alpha_r = atan2(omega * p->lr - vy, vx_eff);
    alpha_f = orc_clamp(alpha_f, -p->maxAlpha, p->maxAlpha);
    alpha_r = orc_clamp(alpha_r, -p->maxAlpha, p->maxAlpha);
    double Fy_f = p->Df * tire_sin(p->Cf * atan(p->Bf * alpha_f));
    double Fy_r = p->Dr * tire_sin(p->Cr * atan(p->Br * alpha_r));
    double Frx = (p->Cm1 - p->Cm2 * vx) * d - p->Cr0 - p->Cr2 * (vx * vx);
    out[0] = Fy_f; out[1] = Fy_r; out[2] = Frx;
}

/* mpc_6stati.py:55-71 */
void orc_f_cont(const orc_params* p, const double x[6], const double u[2], double xdot[6]) {
    double phi = x[2], vx = x[3], vy = x[4], omega = x[5];
    double delta = u[1];
    double m = p->m, Iz = p->Iz, lf = p->lf, lr = p->lr;
    double F[3];
    orc_tire_forces(p, x, u, F);
    double Fy_f = F[0], Fy_r = F[1], Frx = F[2];
    double cphi = cos(phi), sphi = sin(phi);
    double sd = sin(delta), cd = cos(delta);
    xdot[0] = vx * cphi - vy * sphi;
    xdot[1] = vx * sphi + vy * cphi;
    xdot[2] = omega;
    xdot[3] = (1.0 / m) * (Frx - Fy_f * sd + m * vy * omega);
    xdot[4] = (1.0 / m) * (Fy_r + Fy_f * cd - m * vx * omega);
    xdot[5] = (1.0 / Iz) * (Fy_f * lf * cd - Fy_r * lr);
}

/* mpc_6stati.py:73-97 (central differences, columns x then u, then f(x,u)) */
void orc_numerical_jacobian(const orc_params* p, const double x[6], const double u[2], double eps_x,
                            double eps_u, double Jx[36], double Ju[12], double f[6]) {
    double xp[6], xm[6], up[2], um[2], fp[6], fm[6];
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) {
            double dx = (j == i) ? eps_x : 0.0;
            xp[j] = x[j] + dx;
            xm[j] = x[j] - dx;
        }
        orc_f_cont(p, xp, u, fp);
        orc_f_cont(p, xm, u, fm);
        for (int r = 0; r < 6; ++r) Jx[r * 6 + i] = (fp[r] - fm[r]) / (2.0 * eps_x);
    }
    for (int i = 0; i < 2; ++i) {
        for (int j = 0; j < 2; ++j) {
            double du = (j == i) ? eps_u : 0.0;
            up[j] = u[j] + du;
            um[j] = u[j] - du;
        }
        orc_f_cont(p, x, up, fp);
        orc_f_cont(p, x, um, fm);
        for (int r = 0; r < 6; ++r) Ju[r * 2 + i] = (fp[r] - fm[r]) / (2.0 * eps_u);
    }
    orc_f_cont(p, x, u, f);
}

/* mpc_6stati.py:99-109 */
void orc_linearize_discretize(const orc_params* p, const double xbar[6], const double ubar[2], double Ts,
                              double Ad[36], double Bd[12], double g[6]) {
    double Jx[36], Ju[12], f[6];
    orc_numerical_jacobian(p, xbar, ubar, 1e-5, 1e-5, Jx, Ju, f);
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 6; ++c) Ad[r * 6 + c] = ((r == c) ? 1.0 : 0.0) + Ts * Jx[r * 6 + c];
    for (int i = 0; i < 12; ++i) Bd[i] = Ts * Ju[i];
    for (int r = 0; r < 6; ++r) {
        double ax = 0.0, bu = 0.0;
        for (int c = 0; c < 6; ++c) ax += Ad[r * 6 + c] * xbar[c];
        for (int c = 0; c < 2; ++c) bu += Bd[r * 2 + c] * ubar[c];
        g[r] = xbar[r] + Ts * f[r] - ax - bu;
    }
}

/* mpc_6stati.py:111-117 */
double orc_lateral_error(double X, double Y, double Xref, double Yref, double phiref) {
    double s = sin(phiref), c = cos(phiref);
    return s * (X - Xref) - c * (Y - Yref);
}

/* mpc_6stati.py:165-172 */
void orc_nominal_rollout(const orc_params* p, const double x0[6], const double u_prev[2], int N, double Ts,
                         double* xbar) {
    double xk[6], f[6];
    for (int i = 0; i < 6; ++i) { xk[i] = x0[i]; xbar[i * (N + 1)] = x0[i]; }
    for (int k = 0; k < N; ++k) {
        orc_f_cont(p, xk, u_prev, f);
        for (int i = 0; i < 6; ++i) {
            xk[i] = xk[i] + Ts * f[i];
            xbar[i * (N + 1) + k + 1] = xk[i];
        }
    }
}

/* ------------------------------------------------------- dense linear algebra */

/* in-place Cholesky of an SPD n x n row-major matrix (lower factor). returns 0 ok */
static int chol(double* A, int n) {
    for (int j = 0; j < n; ++j) {
        double s = A[j * n + j];
        for (int k = 0; k < j; ++k) s -= A[j * n + k] * A[j * n + k];
        if (!(s > 0.0)) return -1;
        double d = sqrt(s);
        A[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double t = A[i * n + j];
            for (int k = 0; k < j; ++k) t -= A[i * n + k] * A[j * n + k];
            A[i * n + j] = t / d;
        }
    }
    return 0;
}

static void chol_solve(const double* L, int n, double* b) {
    for (int i = 0; i < n; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k];
        b[i] = t / L[i * n + i];
    }
    /* back substitution with each row's terms in descending k: the order in which a column-oriented
     * (lane-parallel) solve produces them, so the GPU's state-bound solver can keep the same arithmetic */
    for (int i = n - 1; i >= 0; --i) {
        double t = b[i];
        for (int k = n - 1; k > i; --k) t -= L[k * n + i] * b[k];
        b[i] = t / L[i * n + i];
    }
}

static double vnorm_inf(const double* v, int n) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) {
        double a = fabs(v[i]);
        if (a > m || a != a) m = a;
    }
    return m;
}

/* ----------------------------------------------------- condensed QP build */
/*
 * Restates the QP of mpc_6stati.py:180-250 over U (2N, stage-major: U_k = u[2k..2k+1])
 * after eliminating X with the dynamics equalities (:187-193):
 *     X_k = xh_k + sum_{j<k} G_{k,j} U_j,  xh_0 = x0, xh_{k+1} = A_k xh_k + g_k.
 * Cost (:217-250):  sum_{k=0}^{N} (C_k X_k - r_k)^T W (C_k X_k - r_k)
 *                   + sum_k U_k^T R U_k + sum_k dU_k^T Rd dU_k
 * with C_k rows [sin phi*_k, -cos phi*_k, 0..], e_phi, e_vx; W = diag(q_c, q_phi, q_vx);
 * r_k = [s Xr - c Yr, phi*_k, vref_k].  In OSQP form: 1/2 u^T P u + q^T u + const.
 * Constraint rows (:195-213), stage-major, 4 per stage: box d, box delta, rate d, rate delta.
 * Optional state rows (:208-213) appended for k = 1..N.
 */
typedef struct {
    int n, m;
    double *P, *q, *A, *l, *u;
    double cst;
    double *Ad, *Bd, *gd;  /* linearization, N stages */
    int infeasible_const;  /* x0 violates state bounds at k=0 */
} qp_t;

static void qp_free(qp_t* qp) {
    free(qp->P); free(qp->q); free(qp->A); free(qp->l); free(qp->u);
    free(qp->Ad); free(qp->Bd); free(qp->gd);
}

static int count_state_rows(const orc_mpc_cfg* c) {
    int r = 0;
    for (int i = 0; i < 6; ++i) {
        double lo = c->has_x_lo ? c->x_lo[i] : -INFINITY;
        double hi = c->has_x_hi ? c->x_hi[i] : INFINITY;
        if (lo > -ORC_INFTY || hi < ORC_INFTY) ++r;
    }
    return r;
}

static void build_qp(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                     const double* path_ref, const double* vref, qp_t* qp) {
    const int N = c->N, n = 2 * N;
    const double Ts = c->Ts;
    const int nsr = count_state_rows(c);
    const int m = 4 * N + nsr * N;
    qp->n = n; qp->m = m;
    qp->P = calloc((size_t)n * n, sizeof(double));
    qp->q = calloc(n, sizeof(double));
    qp->A = calloc((size_t)m * n, sizeof(double));
    qp->l = calloc(m, sizeof(double));
    qp->u = calloc(m, sizeof(double));
    qp->Ad = malloc(sizeof(double) * 36 * N);
    qp->Bd = malloc(sizeof(double) * 12 * N);
    qp->gd = malloc(sizeof(double) * 6 * N);
    qp->infeasible_const = 0;

    /* 1) nominal rollout (:165-172) and 2) linearizations (:175-178) */
    double* xbar = malloc(sizeof(double) * 6 * (N + 1));
    orc_nominal_rollout(p, x0, u_prev, N, Ts, xbar);
    for (int k = 0; k < N; ++k) {
        double xb[6];
        for (int i = 0; i < 6; ++i) xb[i] = xbar[i * (N + 1) + k];
        orc_linearize_discretize(p, xb, u_prev, Ts, qp->Ad + 36 * k, qp->Bd + 12 * k, qp->gd + 6 * k);
    }
    free(xbar);

    /* free response xh and sensitivities G[k][j] (6x2) */
    double* xh = malloc(sizeof(double) * 6 * (N + 1));
    double* G = calloc((size_t)(N + 1) * 6 * n, sizeof(double)); /* G[k] : 6 x n */
    for (int i = 0; i < 6; ++i) xh[i] = x0[i];
    for (int k = 0; k < N; ++k) {
        const double* A = qp->Ad + 36 * k;
        const double* B = qp->Bd + 12 * k;
        const double* g = qp->gd + 6 * k;
        for (int r = 0; r < 6; ++r) {
            double s = 0.0;
            for (int cc = 0; cc < 6; ++cc) s += A[r * 6 + cc] * xh[k * 6 + cc];
            xh[(k + 1) * 6 + r] = s + g[r];
        }
        double* Gk = G + (size_t)k * 6 * n;
        double* Gk1 = G + (size_t)(k + 1) * 6 * n;
        for (int r = 0; r < 6; ++r) {
            for (int j = 0; j < 2 * k; ++j) {
                double s = 0.0;
                for (int cc = 0; cc < 6; ++cc) s += A[r * 6 + cc] * Gk[cc * n + j];
                Gk1[r * n + j] = s;
            }
            Gk1[r * n + 2 * k] = B[r * 2 + 0];
            Gk1[r * n + 2 * k + 1] = B[r * 2 + 1];
        }
    }

    /* tracking cost */
    const double W[3] = {c->q_c, c->q_phi, c->q_vx};
    double cst = 0.0;
    double* F = malloc(sizeof(double) * 3 * n);
    for (int k = 0; k <= N; ++k) {
        double Xr = path_ref[k * 3 + 0], Yr = path_ref[k * 3 + 1], Pr = path_ref[k * 3 + 2];
        double s = sin(Pr), co = cos(Pr);
        const double* xk = xh + 6 * k;
        double e[3];
        e[0] = s * (xk[0] - Xr) - co * (xk[1] - Yr);
        e[1] = xk[2] - Pr;
        e[2] = xk[3] - vref[k];
        for (int t = 0; t < 3; ++t) cst += W[t] * e[t] * e[t];
        if (k == 0) continue;
        const double* Gk = G + (size_t)k * 6 * n;
        for (int j = 0; j < n; ++j) {
            F[0 * n + j] = s * Gk[0 * n + j] - co * Gk[1 * n + j];
            F[1 * n + j] = Gk[2 * n + j];
            F[2 * n + j] = Gk[3 * n + j];
        }
        for (int t = 0; t < 3; ++t)
            for (int i = 0; i < 2 * k; ++i) {
                double wi = 2.0 * W[t] * F[t * n + i];
                qp->q[i] += wi * e[t];
                for (int j = 0; j < 2 * k; ++j) qp->P[i * n + j] += wi * F[t * n + j];
            }
    }
    free(F);

    /* input cost: U^T Rs U, dU^T Rds dU with dU_0 = U_0 - u_prev (:230-240) */
    double Rs[4], Rds[4];
    Rs[0] = c->R[0]; Rs[3] = c->R[3]; Rs[1] = Rs[2] = 0.5 * (c->R[1] + c->R[2]);
    Rds[0] = c->Rd[0]; Rds[3] = c->Rd[3]; Rds[1] = Rds[2] = 0.5 * (c->Rd[1] + c->Rd[2]);
    for (int k = 0; k < N; ++k)
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                qp->P[(2 * k + a) * n + 2 * k + b] += 2.0 * Rs[a * 2 + b];
                /* dU_k = U_k - U_{k-1}: + Rd on (k,k), (k-1,k-1), - Rd on cross terms */
                qp->P[(2 * k + a) * n + 2 * k + b] += 2.0 * Rds[a * 2 + b];
                if (k > 0) {
                    qp->P[(2 * k - 2 + a) * n + 2 * k - 2 + b] += 2.0 * Rds[a * 2 + b];
                    qp->P[(2 * k + a) * n + 2 * k - 2 + b] -= 2.0 * Rds[a * 2 + b];
                    qp->P[(2 * k - 2 + a) * n + 2 * k + b] -= 2.0 * Rds[a * 2 + b];
                }
            }
    for (int a = 0; a < 2; ++a) {
        double t = 0.0;
        for (int b = 0; b < 2; ++b) t += Rds[a * 2 + b] * u_prev[b];
        qp->q[a] -= 2.0 * t;
        cst += u_prev[a] * t;
    }
    qp->cst = cst;

    /* constraints (:195-213) */
    for (int k = 0; k < N; ++k) {
        for (int ch = 0; ch < 2; ++ch) {
            int rb = 4 * k + ch, rr = 4 * k + 2 + ch, j = 2 * k + ch;
            qp->A[(size_t)rb * n + j] = 1.0;
            qp->l[rb] = c->u_lo[ch];
            qp->u[rb] = c->u_hi[ch];
            qp->A[(size_t)rr * n + j] = 1.0;
            if (k > 0) {
                qp->A[(size_t)rr * n + j - 2] = -1.0;
                qp->l[rr] = c->du_lo[ch];
                qp->u[rr] = c->du_hi[ch];
            } else {
                qp->l[rr] = c->du_lo[ch] + u_prev[ch];
                qp->u[rr] = c->du_hi[ch] + u_prev[ch];
            }
        }
    }
    if (nsr > 0) {
        int row = 4 * N;
        for (int i = 0; i < 6; ++i) {
            double lo = c->has_x_lo ? c->x_lo[i] : -INFINITY;
            double hi = c->has_x_hi ? c->x_hi[i] : INFINITY;
            if (!(lo > -ORC_INFTY || hi < ORC_INFTY)) continue;
            if (x0[i] < lo || x0[i] > hi) qp->infeasible_const = 1; /* k = 0: X_0 == x0 */
            for (int k = 1; k <= N; ++k, ++row) {
                const double* Gk = G + (size_t)k * 6 * n;
                for (int j = 0; j < n; ++j) qp->A[(size_t)row * n + j] = Gk[i * n + j];
                qp->l[row] = (lo > -ORC_INFTY) ? lo - xh[6 * k + i] : -INFINITY;
                qp->u[row] = (hi < ORC_INFTY) ? hi - xh[6 * k + i] : INFINITY;
            }
        }
    }
    free(xh);
    free(G);
}

/* interval propagation: exact feasibility test for box + rate rows (chain structure) */
static int box_rate_feasible(const orc_mpc_cfg* c, const double u_prev[2]) {
    for (int ch = 0; ch < 2; ++ch) {
        double lo = u_prev[ch], hi = u_prev[ch];
        for (int k = 0; k < c->N; ++k) {
            double nlo = lo + c->du_lo[ch], nhi = hi + c->du_hi[ch];
            if (nlo < c->u_lo[ch]) nlo = c->u_lo[ch];
            if (nhi > c->u_hi[ch]) nhi = c->u_hi[ch];
            if (!(nlo <= nhi)) return 0;
            lo = nlo; hi = nhi;
        }
    }
    return 1;
}

/* ---------------------------------------------------- OSQP restatement */

typedef struct {
    int n, m;
    double *P, *q, *A, *l, *u;        /* scaled data */
    double *D, *E, *Dinv, *Einv;
    double c, cinv;
    double *rho_vec, *rho_inv;
    double rho;
    double* K;                         /* Cholesky factor of P + sigma I + A^T diag(rho) A */
    double *x, *z, *y, *xt, *zt, *xp, *zp, *yp, *rhs, *tmp_n, *tmp_m, *tmp_m2;
} osqp_ws;

static double limit_scaling(double v) {
    if (v < ORC_MIN_SCALING) return 1.0;
    if (v > ORC_MAX_SCALING) return ORC_MAX_SCALING;
    return v;
}

static void mat_vec(const double* M, int r, int cdim, const double* x, double* y) {
    for (int i = 0; i < r; ++i) {
        double s = 0.0;
        for (int j = 0; j < cdim; ++j) s += M[(size_t)i * cdim + j] * x[j];
        y[i] = s;
    }
}

static void mat_tvec(const double* M, int r, int cdim, const double* x, double* y) {
    for (int j = 0; j < cdim; ++j) y[j] = 0.0;
    for (int i = 0; i < r; ++i) {
        double xi = x[i];
        if (xi == 0.0) continue;
        for (int j = 0; j < cdim; ++j) y[j] += M[(size_t)i * cdim + j] * xi;
    }
}

/* OSQP scale_data (Ruiz equilibration + cost scaling) */
static void osqp_scale(osqp_ws* w, int iters) {
    int n = w->n, m = w->m;
    double* Dt = malloc(sizeof(double) * n);
    double* Et = malloc(sizeof(double) * (m > 0 ? m : 1));
    for (int j = 0; j < n; ++j) w->D[j] = 1.0;
    for (int i = 0; i < m; ++i) w->E[i] = 1.0;
    w->c = 1.0;
    for (int it = 0; it < iters; ++it) {
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int i = 0; i < n; ++i) { double t = fabs(w->P[i * n + j]); if (t > a) a = t; }
            for (int i = 0; i < m; ++i) { double t = fabs(w->A[(size_t)i * n + j]); if (t > a) a = t; }
            Dt[j] = 1.0 / sqrt(limit_scaling(a));
        }
        for (int i = 0; i < m; ++i) {
            double a = 0.0;
            for (int j = 0; j < n; ++j) { double t = fabs(w->A[(size_t)i * n + j]); if (t > a) a = t; }
            Et[i] = 1.0 / sqrt(limit_scaling(a));
        }
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) w->P[i * n + j] *= Dt[i] * Dt[j];
        for (int i = 0; i < m; ++i)
            for (int j = 0; j < n; ++j) w->A[(size_t)i * n + j] *= Et[i] * Dt[j];
        for (int j = 0; j < n; ++j) { w->q[j] *= Dt[j]; w->D[j] *= Dt[j]; }
        for (int i = 0; i < m; ++i) w->E[i] *= Et[i];
        /* cost scaling */
        double mean = 0.0;
        for (int j = 0; j < n; ++j) {
            double a = 0.0;
            for (int i = 0; i < n; ++i) { double t = fabs(w->P[i * n + j]); if (t > a) a = t; }
            mean += a;
        }
        mean /= n;
        double qn = limit_scaling(vnorm_inf(w->q, n));
        double ct = mean > qn ? mean : qn;
        ct = 1.0 / limit_scaling(ct);
        for (int k = 0; k < n * n; ++k) w->P[k] *= ct;
        for (int j = 0; j < n; ++j) w->q[j] *= ct;
        w->c *= ct;
    }
    for (int j = 0; j < n; ++j) w->Dinv[j] = 1.0 / w->D[j];
    for (int i = 0; i < m; ++i) w->Einv[i] = 1.0 / w->E[i];
    w->cinv = 1.0 / w->c;
    for (int i = 0; i < m; ++i) {
        if (w->l[i] > -ORC_INFTY) w->l[i] *= w->E[i]; else w->l[i] = -ORC_INFTY;
        if (w->u[i] < ORC_INFTY) w->u[i] *= w->E[i]; else w->u[i] = ORC_INFTY;
    }
    free(Dt); free(Et);
}

static void set_rho_vec(osqp_ws* w) {
    for (int i = 0; i < w->m; ++i) {
        double r;
        if (w->l[i] <= -ORC_INFTY * ORC_MIN_SCALING && w->u[i] >= ORC_INFTY * ORC_MIN_SCALING) r = ORC_RHO_MIN;
        else if (w->u[i] - w->l[i] < ORC_RHO_TOL) r = ORC_RHO_EQ_OVER_INEQ * w->rho;
        else r = w->rho;
        w->rho_vec[i] = r;
        w->rho_inv[i] = 1.0 / r;
    }
}

/* build + factor M = P + sig I + A^T diag(rv) A (rows with rv == 0 skipped) */
static int factor_kkt(const double* P, const double* A, const double* rv, int n, int m, double sig, double* K) {
    for (int i = 0; i < n * n; ++i) K[i] = P[i];
    for (int i = 0; i < n; ++i) K[i * n + i] += sig;
    for (int r = 0; r < m; ++r) {
        double rr = rv[r];
        if (rr == 0.0) continue;
        const double* a = A + (size_t)r * n;
        for (int i = 0; i < n; ++i) {
            if (a[i] == 0.0) continue;
            double t = rr * a[i];
            for (int j = 0; j < n; ++j) K[i * n + j] += t * a[j];
        }
    }
    return chol(K, n);
}

typedef struct {
    double prim_res, dual_res, eps_prim, eps_dual;
    double ax_n, z_n, px_n, aty_n, q_n;  /* scaled norms for rho estimate */
    double prim_res_s, dual_res_s;
} resid_t;

/* residuals of (x,z,y) in the unscaled problem (OSQP update_info, scaled_termination = 0) */
static void residuals(osqp_ws* w, const orc_mpc_cfg* c, const double* x, const double* z, const double* y,
                      resid_t* r) {
    int n = w->n, m = w->m;
    double* Ax = w->tmp_m;
    double* Px = w->tmp_n;
    double* Aty = malloc(sizeof(double) * n);
    mat_vec(w->A, m, n, x, Ax);
    mat_vec(w->P, n, n, x, Px);
    mat_tvec(w->A, m, n, y, Aty);
    double pr = 0.0, axn = 0.0, zn = 0.0, prs = 0.0, axs = 0.0, zs = 0.0;
    for (int i = 0; i < m; ++i) {
        double d = fabs(w->Einv[i] * (Ax[i] - z[i]));
        if (d > pr) pr = d;
        double t = fabs(w->Einv[i] * Ax[i]); if (t > axn) axn = t;
        t = fabs(w->Einv[i] * z[i]); if (t > zn) zn = t;
        t = fabs(Ax[i] - z[i]); if (t > prs) prs = t;
        t = fabs(Ax[i]); if (t > axs) axs = t;
        t = fabs(z[i]); if (t > zs) zs = t;
    }
    double dr = 0.0, pxn = 0.0, atyn = 0.0, qn = 0.0, drs = 0.0, pxs = 0.0, atys = 0.0, qs = 0.0;
    for (int j = 0; j < n; ++j) {
        double v = Px[j] + w->q[j] + Aty[j];
        double d = fabs(w->Dinv[j] * v) * w->cinv; if (d > dr) dr = d;
        double t = fabs(w->Dinv[j] * Px[j]) * w->cinv; if (t > pxn) pxn = t;
        t = fabs(w->Dinv[j] * Aty[j]) * w->cinv; if (t > atyn) atyn = t;
        t = fabs(w->Dinv[j] * w->q[j]) * w->cinv; if (t > qn) qn = t;
        t = fabs(v); if (t > drs) drs = t;
        t = fabs(Px[j]); if (t > pxs) pxs = t;
        t = fabs(Aty[j]); if (t > atys) atys = t;
        t = fabs(w->q[j]); if (t > qs) qs = t;
    }
    free(Aty);
    r->prim_res = pr;
    r->dual_res = dr;
    r->eps_prim = c->eps_abs + c->eps_rel * (axn > zn ? axn : zn);
    double mx = pxn > atyn ? pxn : atyn; if (qn > mx) mx = qn;
    r->eps_dual = c->eps_abs + c->eps_rel * mx;
    r->prim_res_s = prs; r->dual_res_s = drs;
    r->ax_n = axs; r->z_n = zs; r->px_n = pxs; r->aty_n = atys; r->q_n = qs;
}

/* OSQP is_primal_infeasible (scaled problem, unscaled test) */
static int primal_infeasible(osqp_ws* w, const orc_mpc_cfg* c, const double* dy) {
    int n = w->n, m = w->m;
    double* d = malloc(sizeof(double) * m);
    double nrm = 0.0;
    for (int i = 0; i < m; ++i) {
        double v = dy[i];
        /* project onto the cone of directions admissible for infinite bounds */
        if (w->u[i] >= ORC_INFTY * ORC_MIN_SCALING && v > 0.0) v = 0.0;
        if (w->l[i] <= -ORC_INFTY * ORC_MIN_SCALING && v < 0.0) v = 0.0;
        d[i] = v;
        double t = fabs(w->E[i] * v);
        if (t > nrm) nrm = t;
    }
    int inf = 0;
    if (nrm > ORC_DIV_TOL) {
        double lhs = 0.0;
        for (int i = 0; i < m; ++i) {
            if (d[i] > 0.0) lhs += w->u[i] * d[i];
            else if (d[i] < 0.0) lhs += w->l[i] * d[i];
        }
        if (lhs < -c->eps_prim_inf * nrm) {
            double* Atd = malloc(sizeof(double) * n);
            mat_tvec(w->A, m, n, d, Atd);
            double an = 0.0;
            for (int j = 0; j < n; ++j) { double t = fabs(w->Dinv[j] * Atd[j]); if (t > an) an = t; }
            free(Atd);
            if (an < c->eps_prim_inf * nrm) inf = 1;
        }
    }
    free(d);
    return inf;
}

/* Reduced-KKT solve for a given active set (OSQP polish.c, form_KKT + iterative_refinement), in
 * eliminated form: (P + dI + Ar^T Ar / d) x = r1 + Ar^T r2 / d, y_r = (Ar x - r2) / d, refined
 * polish_refine_iter times against the unregularized KKT [P Ar^T; Ar 0] (x; y_r) = (-q; b).
 * act[i]: -1 lower active (b = l), +1 upper active (b = u), 0 inactive.  Outputs x, y (0 on
 * inactive rows) and Ax.  Returns 1 on success. */
static int kkt_solve_active(osqp_ws* w, const orc_mpc_cfg* c, const int* act, double* x, double* y, double* Ax) {
    int n = w->n, m = w->m;
    double dlt = c->delta;
    int mm = m > 0 ? m : 1;
    double* b = calloc(mm, sizeof(double));
    double* rv = calloc(mm, sizeof(double));
    for (int i = 0; i < m; ++i) {
        if (act[i] < 0) b[i] = w->l[i];
        else if (act[i] > 0) b[i] = w->u[i];
        rv[i] = act[i] ? 1.0 / dlt : 0.0;
    }
    double* K = malloc(sizeof(double) * n * n);
    int ok = factor_kkt(w->P, w->A, rv, n, m, dlt, K) == 0;
    double* r1 = malloc(sizeof(double) * n);
    double* r2 = malloc(sizeof(double) * mm);
    double* t = malloc(sizeof(double) * n);
    if (ok) {
        for (int j = 0; j < n; ++j) { x[j] = 0.0; r1[j] = -w->q[j]; }
        for (int i = 0; i < m; ++i) { y[i] = 0.0; r2[i] = act[i] ? b[i] : 0.0; }
        for (int pass = 0; pass <= c->polish_refine_iter; ++pass) {
            for (int j = 0; j < n; ++j) t[j] = r1[j];
            for (int i = 0; i < m; ++i) {
                if (!act[i]) continue;
                double s = r2[i] / dlt;
                const double* a = w->A + (size_t)i * n;
                for (int j = 0; j < n; ++j) t[j] += a[j] * s;
            }
            chol_solve(K, n, t);
            mat_vec(w->A, m, n, t, Ax);
            for (int j = 0; j < n; ++j) x[j] += t[j];
            for (int i = 0; i < m; ++i)
                if (act[i]) y[i] += (Ax[i] - r2[i]) / dlt;
            if (pass == c->polish_refine_iter) break;
            mat_vec(w->P, n, n, x, r1);
            mat_tvec(w->A, m, n, y, t);
            for (int j = 0; j < n; ++j) r1[j] = -w->q[j] - r1[j] - t[j];
            mat_vec(w->A, m, n, x, Ax);
            for (int i = 0; i < m; ++i) r2[i] = act[i] ? b[i] - Ax[i] : 0.0;
        }
        mat_vec(w->A, m, n, x, Ax);
    }
    free(b); free(rv); free(K); free(r1); free(r2); free(t);
    return ok;
}

/* OSQP active-set rule (polish.c form_Ared): lower if z - l < -y, upper if u - z < y */
static void active_set(const osqp_ws* w, const double* z, const double* y, int* act) {
    for (int i = 0; i < w->m; ++i) {
        act[i] = 0;
        if (z[i] - w->l[i] < -y[i]) act[i] = -1;
        else if (w->u[i] - z[i] < y[i]) act[i] = 1;
    }
}

/* OSQP polish: one reduced solve, then (z, y) projected onto the normal cone (project_normalcone). */
static int osqp_polish(osqp_ws* w, const orc_mpc_cfg* c, double* xo, double* zo, double* yo, resid_t* rpol) {
    int m = w->m, mm = m > 0 ? m : 1;
    int* act = malloc(sizeof(int) * mm);
    double* Ax = malloc(sizeof(double) * mm);
    double* yr = malloc(sizeof(double) * mm);
    active_set(w, w->z, w->y, act);
    int ok = kkt_solve_active(w, c, act, xo, yr, Ax);
    if (ok) {
        for (int i = 0; i < m; ++i) {
            double zt = Ax[i] + yr[i];
            double zz = zt < w->l[i] ? w->l[i] : (zt > w->u[i] ? w->u[i] : zt);
            zo[i] = zz;
            yo[i] = zt - zz;
        }
        residuals(w, c, xo, zo, yo, rpol);
    }
    free(act); free(Ax); free(yr);
    return ok;
}

/* Exact polish: the reduced solve iterated as a primal-dual active-set method.  After each solve the
 * KKT conditions of the unscaled problem are checked -- stationarity, primal feasibility and
 * multiplier signs (y <= 0 on lower-active rows, y >= 0 on upper-active rows), each to cert_tol
 * relative to the problem's own scale; if they hold the point is the QP optimum and is returned.
 * Otherwise the OSQP active-set rule is re-applied to the polished (Ax, y) and the solve repeats. */
static int exact_polish(osqp_ws* w, const orc_mpc_cfg* c, double* xo, double* zo, double* yo, int* passes) {
    int n = w->n, m = w->m, mm = m > 0 ? m : 1;
    int* act = malloc(sizeof(int) * mm);
    double* Ax = malloc(sizeof(double) * mm);
    double* y = malloc(sizeof(double) * mm);
    double* x = malloc(sizeof(double) * n);
    double* Px = malloc(sizeof(double) * n);
    double* Aty = malloc(sizeof(double) * n);
    active_set(w, w->z, w->y, act);
    int cert = 0, pass;
    const double tol = c->cert_tol;
    for (pass = 1; pass <= c->polish_max_pass; ++pass) {
        if (!kkt_solve_active(w, c, act, x, y, Ax)) break;
        /* certificate (unscaled quantities) */
        mat_vec(w->P, n, n, x, Px);
        mat_tvec(w->A, m, n, y, Aty);
        double st = 0.0, gsc = 1.0;
        for (int j = 0; j < n; ++j) {
            double v = fabs(w->Dinv[j] * (Px[j] + w->q[j] + Aty[j])) * w->cinv;
            if (v > st) st = v;
            double s1 = fabs(w->Dinv[j] * w->q[j]) * w->cinv; if (s1 > gsc) gsc = s1;
            s1 = fabs(w->Dinv[j] * Px[j]) * w->cinv; if (s1 > gsc) gsc = s1;
        }
        int okc = st <= tol * gsc;
        for (int i = 0; i < m && okc; ++i) {
            double ax = Ax[i] * w->Einv[i];
            if (w->l[i] > -ORC_INFTY) { double lo = w->l[i] * w->Einv[i]; if (ax < lo - tol * (1.0 + fabs(lo))) okc = 0; }
            if (w->u[i] < ORC_INFTY) { double hi = w->u[i] * w->Einv[i]; if (ax > hi + tol * (1.0 + fabs(hi))) okc = 0; }
            double yu = y[i] * w->E[i] * w->cinv;
            if (act[i] < 0 && yu > tol * gsc) okc = 0;
            if (act[i] > 0 && yu < -tol * gsc) okc = 0;
        }
        if (okc) { cert = 1; break; }
        active_set(w, Ax, y, act);
    }
    if (cert) {
        memcpy(xo, x, sizeof(double) * n);
        for (int i = 0; i < m; ++i) {
            double zz = Ax[i] < w->l[i] ? w->l[i] : (Ax[i] > w->u[i] ? w->u[i] : Ax[i]);
            zo[i] = zz;
            yo[i] = y[i];
        }
    }
    *passes = pass;
    free(act); free(Ax); free(y); free(x); free(Px); free(Aty);
    return cert;
}

/* Solve the scaled QP; returns status; x (unscaled) in xout */
static int osqp_solve(qp_t* qp, const orc_mpc_cfg* c, double* xout, orc_info* info, orc_warm* warm) {
    int n = qp->n, m = qp->m;
    osqp_ws w;
    memset(&w, 0, sizeof(w));
    w.n = n; w.m = m;
    w.P = malloc(sizeof(double) * n * n); memcpy(w.P, qp->P, sizeof(double) * n * n);
    w.q = malloc(sizeof(double) * n); memcpy(w.q, qp->q, sizeof(double) * n);
    w.A = malloc(sizeof(double) * (size_t)m * n); memcpy(w.A, qp->A, sizeof(double) * (size_t)m * n);
    w.l = malloc(sizeof(double) * m); memcpy(w.l, qp->l, sizeof(double) * m);
    w.u = malloc(sizeof(double) * m); memcpy(w.u, qp->u, sizeof(double) * m);
    w.D = malloc(sizeof(double) * n); w.Dinv = malloc(sizeof(double) * n);
    w.E = malloc(sizeof(double) * m); w.Einv = malloc(sizeof(double) * m);
    w.rho_vec = malloc(sizeof(double) * m); w.rho_inv = malloc(sizeof(double) * m);
    w.K = malloc(sizeof(double) * n * n);
    double** vn[] = {&w.x, &w.xt, &w.xp, &w.rhs, &w.tmp_n};
    for (size_t i = 0; i < sizeof(vn) / sizeof(vn[0]); ++i) *vn[i] = calloc(n, sizeof(double));
    double** vm[] = {&w.z, &w.y, &w.zt, &w.zp, &w.yp, &w.tmp_m, &w.tmp_m2};
    for (size_t i = 0; i < sizeof(vm) / sizeof(vm[0]); ++i) *vm[i] = calloc(m, sizeof(double));

    int status = ORC_SOLVER_ERROR;
    w.rho = c->rho;
    if (c->scaling_iters > 0) osqp_scale(&w, c->scaling_iters);
    else {
        for (int j = 0; j < n; ++j) w.D[j] = w.Dinv[j] = 1.0;
        for (int i = 0; i < m; ++i) w.E[i] = w.Einv[i] = 1.0;
        w.c = w.cinv = 1.0;
    }
    if (warm && warm->valid)   /* start from the previous step's adapted rho (x = z = y = 0 as cold) */
        w.rho = warm->rho < ORC_RHO_MIN ? ORC_RHO_MIN : (warm->rho > ORC_RHO_MAX ? ORC_RHO_MAX : warm->rho);
    set_rho_vec(&w);
    if (factor_kkt(w.P, w.A, w.rho_vec, n, m, c->sigma, w.K) != 0) goto done;

    resid_t r = {0};
    int iter = 1, converged = 0, rounds = 0;
    double escale = 1.0;   /* exact mode: tolerance tightening between polish attempts */
admm_loop:
    for (; iter <= c->max_iter; ++iter) {
        memcpy(w.xp, w.x, sizeof(double) * n);
        memcpy(w.zp, w.z, sizeof(double) * m);
        memcpy(w.yp, w.y, sizeof(double) * m);
        /* update_xz_tilde */
        for (int i = 0; i < m; ++i) w.tmp_m2[i] = w.rho_vec[i] * w.zp[i] - w.y[i];
        mat_tvec(w.A, m, n, w.tmp_m2, w.rhs);
        for (int j = 0; j < n; ++j) w.rhs[j] += c->sigma * w.xp[j] - w.q[j];
        memcpy(w.xt, w.rhs, sizeof(double) * n);
        chol_solve(w.K, n, w.xt);
        mat_vec(w.A, m, n, w.xt, w.zt);
        /* update_x, update_z, update_y */
        for (int j = 0; j < n; ++j) w.x[j] = c->alpha * w.xt[j] + (1.0 - c->alpha) * w.xp[j];
        for (int i = 0; i < m; ++i) {
            double zr = c->alpha * w.zt[i] + (1.0 - c->alpha) * w.zp[i];
            double v = zr + w.rho_inv[i] * w.y[i];
            double zz = v < w.l[i] ? w.l[i] : (v > w.u[i] ? w.u[i] : v);
            w.z[i] = zz;
            w.y[i] = w.y[i] + w.rho_vec[i] * (zr - zz);
        }
        int check = (iter % c->check_interval == 0);
        if (check) {
            residuals(&w, c, w.x, w.z, w.y, &r);
            if (r.prim_res <= escale * r.eps_prim && r.dual_res <= escale * r.eps_dual) { converged = 1; break; }
            double* dy = w.tmp_m2;
            for (int i = 0; i < m; ++i) dy[i] = w.y[i] - w.yp[i];
            if (primal_infeasible(&w, c, dy)) { status = ORC_INFEASIBLE; goto done_iter; }
        }
        if (c->adaptive_rho && (iter % c->check_interval == 0)) {
            double pn = r.ax_n > r.z_n ? r.ax_n : r.z_n;
            double dn = r.px_n > r.aty_n ? r.px_n : r.aty_n; if (r.q_n > dn) dn = r.q_n;
            double pr = r.prim_res_s / (pn + ORC_DIV_TOL);
            double dr = r.dual_res_s / (dn + ORC_DIV_TOL);
            double est = w.rho * sqrt(pr / (dr + ORC_DIV_TOL));
            if (est < ORC_RHO_MIN) est = ORC_RHO_MIN;
            if (est > ORC_RHO_MAX) est = ORC_RHO_MAX;
            if (est > w.rho * c->adaptive_rho_tol || est < w.rho / c->adaptive_rho_tol) {
                w.rho = est;
                set_rho_vec(&w);
                if (factor_kkt(w.P, w.A, w.rho_vec, n, m, c->sigma, w.K) != 0) { status = ORC_SOLVER_ERROR; goto done_iter; }
            }
        }
    }
    if (converged) status = ORC_OPTIMAL;
    else {
        iter = c->max_iter;
        residuals(&w, c, w.x, w.z, w.y, &r);
        if (rounds > 0 && r.prim_res <= r.eps_prim && r.dual_res <= r.eps_dual)
            status = ORC_OPTIMAL;   /* exact-mode continuation ran out of iterations: eps still met */
        else if (r.prim_res <= 10.0 * r.eps_prim && r.dual_res <= 10.0 * r.eps_dual) status = ORC_OPTIMAL_INACCURATE;
        else status = ORC_USER_LIMIT;
    }
    info->polished = 0;
    if (status == ORC_OPTIMAL && c->polish && c->polish_mode == 1) {
        double* xpol = malloc(sizeof(double) * n);
        double* zpol = malloc(sizeof(double) * (m > 0 ? m : 1));
        double* ypol = malloc(sizeof(double) * (m > 0 ? m : 1));
        int passes = 0;
        if (exact_polish(&w, c, xpol, zpol, ypol, &passes)) {
            memcpy(w.x, xpol, sizeof(double) * n);
            memcpy(w.z, zpol, sizeof(double) * m);
            memcpy(w.y, ypol, sizeof(double) * m);
            residuals(&w, c, w.x, w.z, w.y, &r);
            info->polished = passes + 16 * rounds;
        }
        free(xpol); free(zpol); free(ypol);
        if (!info->polished && rounds < c->polish_max_rounds && iter < c->max_iter) {
            /* not certified: continue ADMM to a 100x tighter tolerance and polish again */
            ++rounds;
            escale *= 1e-2;
            converged = 0;
            ++iter;
            goto admm_loop;
        }
    } else if (status == ORC_OPTIMAL && c->polish) {
        double* xpol = malloc(sizeof(double) * n);
        double* zpol = malloc(sizeof(double) * (m > 0 ? m : 1));
        double* ypol = malloc(sizeof(double) * (m > 0 ? m : 1));
        resid_t rp;
        if (osqp_polish(&w, c, xpol, zpol, ypol, &rp)) {
            int ok = (rp.prim_res < r.prim_res && rp.dual_res < r.dual_res) ||
                     (rp.prim_res < r.prim_res && r.dual_res < 1e-10) ||
                     (rp.dual_res < r.dual_res && r.prim_res < 1e-10);
            if (ok) {
                memcpy(w.x, xpol, sizeof(double) * n);
                memcpy(w.z, zpol, sizeof(double) * m);
                memcpy(w.y, ypol, sizeof(double) * m);
                r = rp;
                info->polished = 1;
            }
        }
        free(xpol); free(zpol); free(ypol);
    }
done_iter:
    info->iters = iter > c->max_iter ? c->max_iter : iter;
    info->prim_res = r.prim_res;
    info->dual_res = r.dual_res;
    info->rho_final = w.rho;
    for (int j = 0; j < n; ++j) xout[j] = w.D[j] * w.x[j];
    if (warm) {
        warm->rho = w.rho;
        warm->valid = (status == ORC_OPTIMAL || status == ORC_OPTIMAL_INACCURATE);
    }
done:
    free(w.P); free(w.q); free(w.A); free(w.l); free(w.u); free(w.D); free(w.Dinv); free(w.E); free(w.Einv);
    free(w.rho_vec); free(w.rho_inv); free(w.K);
    free(w.x); free(w.xt); free(w.xp); free(w.rhs); free(w.tmp_n);
    free(w.z); free(w.y); free(w.zt); free(w.zp); free(w.yp); free(w.tmp_m); free(w.tmp_m2);
    return status;
}

/* cost of mpc_6stati.py:217-250 evaluated at (X, U): X (6,N+1), U (2,N) row-major */
static double eval_cost(const orc_mpc_cfg* c, const double x0[6], const double u_prev[2], const double* path_ref,
                        const double* vref, const double* X, const double* U) {
    int N = c->N;
    double obj = 0.0;
    (void)x0;
    for (int k = 0; k <= N; ++k) {
        double ec = orc_lateral_error(X[0 * (N + 1) + k], X[1 * (N + 1) + k], path_ref[3 * k], path_ref[3 * k + 1],
                                      path_ref[3 * k + 2]);
        double ep = X[2 * (N + 1) + k] - path_ref[3 * k + 2];
        double ev = X[3 * (N + 1) + k] - vref[k];
        obj += c->q_c * ec * ec + c->q_phi * ep * ep + c->q_vx * ev * ev;
        if (k == N) break;
        double uk[2] = {U[k], U[N + k]};
        double du[2];
        for (int a = 0; a < 2; ++a) du[a] = uk[a] - (k == 0 ? u_prev[a] : U[a * N + k - 1]);
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) obj += uk[a] * c->R[a * 2 + b] * uk[b] + du[a] * c->Rd[a * 2 + b] * du[b];
    }
    return obj;
}

static int all_finite(const double* v, int n) {
    for (int i = 0; i < n; ++i)
        if (!isfinite(v[i])) return 0;
    return 1;
}

/* mpc_6stati.py:120-275 */
int orc_mpc_step(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                 const double* path_ref, const double* vref, double u_cmd[2], double* X_opt, double* U_opt,
                 orc_info* info) {
    return orc_mpc_step_warm(p, c, x0, u_prev, path_ref, vref, u_cmd, X_opt, U_opt, info, NULL);
}

/* The QP half by the structured IPM (riccati_ipm.c) on the sparse form, linearization given. */
int orc_qp_ipm(const orc_mpc_cfg* c, const double x0[6], const double u_prev[2], const double* path_ref,
               const double* vref, const double* Ad, const double* Bd, const double* gd, const double* xinit,
               double* U_opt, double* X_opt, orc_info* info) {
    const int N = c->N;
    orc_info dummy;
    if (!info) info = &dummy;
    memset(info, 0, sizeof(*info));
    info->polished = -1;
    info->objective = NAN;
    if (!all_finite(x0, 6) || !all_finite(u_prev, 2) || !all_finite(path_ref, 3 * (N + 1)) ||
        !all_finite(vref, N + 1) || !all_finite(Ad, 36 * N) || !all_finite(Bd, 12 * N) || !all_finite(gd, 6 * N)) {
        info->status = ORC_SOLVER_ERROR;
        return info->status;
    }
    if (!box_rate_feasible(c, u_prev)) {
        info->status = ORC_INFEASIBLE;
        return info->status;
    }
    double* Q = malloc(sizeof(double) * 36 * (N + 1));
    double* qv = malloc(sizeof(double) * 6 * (N + 1));
    double* X = malloc(sizeof(double) * 6 * (N + 1));
    double* U = malloc(sizeof(double) * 2 * N);
    double res[5];
    orc_ipm_state_cost(c, path_ref, vref, Q, qv);
    int it = 0;
    const int st = orc_ipm_core(c, N, x0, u_prev, Q, qv, Ad, Bd, gd, xinit, X, U, &it, res);
    info->status = st;
    info->iters = it;
    info->prim_res = res[0] > res[1] ? res[0] : res[1];
    info->dual_res = res[2];
    if (st == ORC_OPTIMAL || st == ORC_OPTIMAL_INACCURATE) {
        double* Xr = malloc(sizeof(double) * 6 * (N + 1));
        double* Ur = malloc(sizeof(double) * 2 * N);
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 6; ++i) Xr[i * (N + 1) + k] = X[6 * k + i];
        for (int k = 0; k < N; ++k) { Ur[k] = U[2 * k]; Ur[N + k] = U[2 * k + 1]; }
        info->objective = eval_cost(c, x0, u_prev, path_ref, vref, Xr, Ur);
        if (X_opt) memcpy(X_opt, Xr, sizeof(double) * 6 * (N + 1));
        if (U_opt) memcpy(U_opt, Ur, sizeof(double) * 2 * N);
        free(Xr); free(Ur);
    }
    free(Q); free(qv); free(X); free(U);
    return st;
}

int orc_mpc_step_warm(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                      const double* path_ref, const double* vref, double u_cmd[2], double* X_opt, double* U_opt,
                      orc_info* info, orc_warm* warm) {
    int N = c->N, n = 2 * N;
    orc_info dummy;
    if (!info) info = &dummy;
    memset(info, 0, sizeof(*info));
    u_cmd[0] = u_prev[0]; u_cmd[1] = u_prev[1];   /* fallback (:257-262) */
    if (!all_finite(x0, 6) || !all_finite(u_prev, 2) || !all_finite(path_ref, 3 * (N + 1)) ||
        !all_finite(vref, N + 1)) {
        info->status = ORC_SOLVER_ERROR;
        return info->status;
    }
    if (c->solver == 2 || (c->solver == 0 && N >= ORC_IPM_AUTO_MIN_N)) {
        /* structured IPM on the sparse form: nominal rollout + linearization (:165-178), then the QP */
        double* xbar = malloc(sizeof(double) * 6 * (N + 1));
        double* xin = malloc(sizeof(double) * 6 * (N + 1));
        double *Ad = malloc(sizeof(double) * 36 * N), *Bd = malloc(sizeof(double) * 12 * N),
               *gd = malloc(sizeof(double) * 6 * N);
        orc_nominal_rollout(p, x0, u_prev, N, c->Ts, xbar);
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 6; ++i) xin[6 * k + i] = xbar[i * (N + 1) + k];
        for (int k = 0; k < N; ++k)
            orc_linearize_discretize(p, xin + 6 * k, u_prev, c->Ts, Ad + 36 * k, Bd + 12 * k, gd + 6 * k);
        double* U = malloc(sizeof(double) * 2 * N);
        const int st = orc_qp_ipm(c, x0, u_prev, path_ref, vref, Ad, Bd, gd, xin, U, X_opt, info);
        if (st == ORC_OPTIMAL || st == ORC_OPTIMAL_INACCURATE) {
            u_cmd[0] = U[0]; u_cmd[1] = U[N];
            if (U_opt) memcpy(U_opt, U, sizeof(double) * 2 * N);
        }
        if (warm) warm->valid = 0;
        free(xbar); free(xin); free(Ad); free(Bd); free(gd); free(U);
        return st;
    }
    qp_t qp;
    build_qp(p, c, x0, u_prev, path_ref, vref, &qp);
    int st;
    double* u = calloc(n, sizeof(double));
    if (!all_finite(qp.P, n * n) || !all_finite(qp.q, n) || !all_finite(qp.A, qp.m * n)) {
        st = ORC_SOLVER_ERROR;
    } else if (qp.infeasible_const || !box_rate_feasible(c, u_prev)) {
        st = ORC_INFEASIBLE;
    } else {
        st = osqp_solve(&qp, c, u, info, warm);
    }
    info->status = st;
    if ((c->solver == 0 || c->solver == 3) && (st == ORC_SOLVER_ERROR || st == ORC_USER_LIMIT)) {
        /* the condensed problem failed numerically (non-finite condensed data, a failed KKT
         * factorization, no convergence): solve the sparse form by the structured IPM instead */
        double* xbar = malloc(sizeof(double) * 6 * (N + 1));
        double* xin = malloc(sizeof(double) * 6 * (N + 1));
        double* U = malloc(sizeof(double) * 2 * N);
        orc_nominal_rollout(p, x0, u_prev, N, c->Ts, xbar);
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < 6; ++i) xin[6 * k + i] = xbar[i * (N + 1) + k];
        st = orc_qp_ipm(c, x0, u_prev, path_ref, vref, qp.Ad, qp.Bd, qp.gd, xin, U, X_opt, info);
        if (st == ORC_OPTIMAL || st == ORC_OPTIMAL_INACCURATE) {
            u_cmd[0] = U[0]; u_cmd[1] = U[N];
            if (U_opt) memcpy(U_opt, U, sizeof(double) * 2 * N);
        }
        if (warm) warm->valid = 0;
        free(xbar); free(xin); free(U); free(u);
        qp_free(&qp);
        return st;
    }
    if (warm && st != ORC_OPTIMAL && st != ORC_OPTIMAL_INACCURATE) warm->valid = 0;
    if (st == ORC_OPTIMAL || st == ORC_OPTIMAL_INACCURATE) {
        double* X = malloc(sizeof(double) * 6 * (N + 1));
        double* U = malloc(sizeof(double) * 2 * N);
        for (int k = 0; k < N; ++k) { U[k] = u[2 * k]; U[N + k] = u[2 * k + 1]; }
        for (int i = 0; i < 6; ++i) X[i * (N + 1)] = x0[i];
        for (int k = 0; k < N; ++k) {
            const double* A = qp.Ad + 36 * k;
            const double* B = qp.Bd + 12 * k;
            const double* g = qp.gd + 6 * k;
            for (int r = 0; r < 6; ++r) {
                double s = 0.0;
                for (int cc = 0; cc < 6; ++cc) s += A[r * 6 + cc] * X[cc * (N + 1) + k];
                s += B[r * 2] * U[k] + B[r * 2 + 1] * U[N + k] + g[r];
                X[r * (N + 1) + k + 1] = s;
            }
        }
        info->objective = eval_cost(c, x0, u_prev, path_ref, vref, X, U);
        u_cmd[0] = U[0]; u_cmd[1] = U[N];
        if (X_opt) memcpy(X_opt, X, sizeof(double) * 6 * (N + 1));
        if (U_opt) memcpy(U_opt, U, sizeof(double) * 2 * N);
        free(X); free(U);
    } else {
        info->objective = NAN;
    }
    free(u);
    qp_free(&qp);
    return st;
}

void orc_mpc_step_batch(const orc_params* p, const orc_mpc_cfg* c, int B, const double* x0,
                        const double* u_prev, const double* path_ref, const double* vref, double* u_cmd,
                        int* status, double* objective, double* X_opt, double* U_opt, int* iters,
                        int* polished, int nthreads) {
    int N = c->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int b = 0; b < B; ++b) {
        orc_info info;
        int st = orc_mpc_step(p, c, x0 + 6 * b, u_prev + 2 * b, path_ref + (size_t)3 * (N + 1) * b,
                              vref + (size_t)(N + 1) * b, u_cmd + 2 * b,
                              X_opt ? X_opt + (size_t)6 * (N + 1) * b : NULL,
                              U_opt ? U_opt + (size_t)2 * N * b : NULL, &info);
        if (status) status[b] = st;
        if (objective) objective[b] = info.objective;
        if (iters) iters[b] = info.iters;
        if (polished) polished[b] = info.polished;
    }
}

/* orc_mpc_step_batch with a warm start per instance (the closed loop's carried rho, MPC/main.py's loop calling
 * mpc_6stati.py:252-256 with warm_start=True): rho[b] / valid[b] are read as the instance's orc_warm and written
 * back after its solve. */
void orc_mpc_step_batch_warm(const orc_params* p, const orc_mpc_cfg* c, int B, const double* x0,
                             const double* u_prev, const double* path_ref, const double* vref, double* rho,
                             int* valid, double* u_cmd, int* status, int* iters, int* polished, int nthreads) {
    int N = c->N;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 4)
#endif
    for (int b = 0; b < B; ++b) {
        orc_info info;
        orc_warm w = {valid[b], rho[b]};
        int st = orc_mpc_step_warm(p, c, x0 + 6 * b, u_prev + 2 * b, path_ref + (size_t)3 * (N + 1) * b,
                                   vref + (size_t)(N + 1) * b, u_cmd + 2 * b, NULL, NULL, &info, &w);
        rho[b] = w.rho;
        valid[b] = w.valid;
        if (status) status[b] = st;
        if (iters) iters[b] = info.iters;
        if (polished) polished[b] = info.polished;
    }
}

/* ------------------------------------------- exact QP (validation solver) */
/* Dense primal-dual interior point (Mehrotra) on the condensed QP:  min 1/2 u'Pu + q'u  s.t.  l <= A u <= u,
 * as one-sided rows G u <= h.  Independent of the ADMM path; used by tests to certify it. */
int orc_qp_exact(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                 const double* path_ref, const double* vref, double* U_opt, double* objective) {
    qp_t qp;
    build_qp(p, c, x0, u_prev, path_ref, vref, &qp);
    int n = qp.n, m = qp.m, N = c->N;
    int mg = 0;
    for (int i = 0; i < m; ++i) { if (qp.u[i] < ORC_INFTY) ++mg; if (qp.l[i] > -ORC_INFTY) ++mg; }
    double* G = calloc((size_t)mg * n, sizeof(double));
    double* h = malloc(sizeof(double) * mg);
    int r = 0;
    for (int i = 0; i < m; ++i) {
        if (qp.u[i] < ORC_INFTY) { for (int j = 0; j < n; ++j) G[(size_t)r * n + j] = qp.A[(size_t)i * n + j]; h[r++] = qp.u[i]; }
        if (qp.l[i] > -ORC_INFTY) { for (int j = 0; j < n; ++j) G[(size_t)r * n + j] = -qp.A[(size_t)i * n + j]; h[r++] = -qp.l[i]; }
    }
    double *x = calloc(n, sizeof(double)), *s = malloc(sizeof(double) * mg), *lam = malloc(sizeof(double) * mg);
    double *rd = malloc(sizeof(double) * n), *rp = malloc(sizeof(double) * mg), *Gx = malloc(sizeof(double) * mg);
    double *dx = malloc(sizeof(double) * n), *ds = malloc(sizeof(double) * mg), *dl = malloc(sizeof(double) * mg);
    double *K = malloc(sizeof(double) * n * n), *w = malloc(sizeof(double) * mg), *rhs = malloc(sizeof(double) * n);
    double *tmp = malloc(sizeof(double) * n);
    int ret = -1;
    /* start: x = 0, s = max(h - Gx, 1), lam = 1 */
    for (int i = 0; i < mg; ++i) { s[i] = h[i] > 1.0 ? h[i] : 1.0; lam[i] = 1.0; }
    for (int it = 0; it < 200; ++it) {
        /* residuals: rd = Px + q + G'lam ; rp = Gx + s - h */
        mat_vec(qp.P, n, n, x, rd);
        mat_tvec(G, mg, n, lam, tmp);
        for (int j = 0; j < n; ++j) rd[j] += qp.q[j] + tmp[j];
        mat_vec(G, mg, n, x, Gx);
        double mu = 0.0;
        for (int i = 0; i < mg; ++i) { rp[i] = Gx[i] + s[i] - h[i]; mu += s[i] * lam[i]; }
        mu /= (mg > 0 ? mg : 1);
        double rdn = vnorm_inf(rd, n), rpn = vnorm_inf(rp, mg);
        if (rdn < 1e-10 * (1.0 + vnorm_inf(qp.q, n)) && rpn < 1e-11 && mu < 1e-13) { ret = 0; break; }
        /* K = P + G' diag(lam/s) G */
        for (int i = 0; i < n * n; ++i) K[i] = qp.P[i];
        for (int i = 0; i < mg; ++i) {
            w[i] = lam[i] / s[i];
            const double* g = G + (size_t)i * n;
            for (int a = 0; a < n; ++a) {
                if (g[a] == 0.0) continue;
                double t = w[i] * g[a];
                for (int b = 0; b < n; ++b) K[a * n + b] += t * g[b];
            }
        }
        if (chol(K, n) != 0) break;
        double alpha_aff = 1.0, sigma = 0.0;
        for (int pass = 0; pass < 2; ++pass) {
            /* complementarity target: s*lam = sigma*mu - ds_aff*dl_aff (corrector) */
            /* solve: P dx + G' dl = -rd ; G dx + ds = -rp ; lam ds + s dl = -s lam + t */
            for (int j = 0; j < n; ++j) rhs[j] = -rd[j];
            double* rc = malloc(sizeof(double) * mg);
            for (int i = 0; i < mg; ++i) {
                double t = (pass == 0) ? 0.0 : sigma * mu - ds[i] * dl[i];
                rc[i] = -s[i] * lam[i] + t;
                /* eliminate: dl = (rc - lam ds)/s, ds = -rp - G dx  => dl = (rc + lam(rp + G dx))/s */
                double coef = (rc[i] + lam[i] * rp[i]) / s[i];
                const double* g = G + (size_t)i * n;
                for (int j = 0; j < n; ++j) rhs[j] -= g[j] * coef;
            }
            chol_solve(K, n, rhs);
            memcpy(dx, rhs, sizeof(double) * n);
            mat_vec(G, mg, n, dx, Gx);
            for (int i = 0; i < mg; ++i) {
                ds[i] = -rp[i] - Gx[i];
                dl[i] = (rc[i] - lam[i] * ds[i]) / s[i];
            }
            free(rc);
            double a = 1.0;
            for (int i = 0; i < mg; ++i) {
                if (ds[i] < 0.0) { double t = -s[i] / ds[i]; if (t < a) a = t; }
                if (dl[i] < 0.0) { double t = -lam[i] / dl[i]; if (t < a) a = t; }
            }
            if (pass == 0) {
                alpha_aff = a;
                double mu_aff = 0.0;
                for (int i = 0; i < mg; ++i) mu_aff += (s[i] + a * ds[i]) * (lam[i] + a * dl[i]);
                mu_aff /= (mg > 0 ? mg : 1);
                sigma = pow(mu_aff / mu, 3.0);
            } else {
                a *= 0.99;
                if (a > 1.0) a = 1.0;
                for (int j = 0; j < n; ++j) x[j] += a * dx[j];
                for (int i = 0; i < mg; ++i) { s[i] += a * ds[i]; lam[i] += a * dl[i]; }
            }
        }
        (void)alpha_aff;
    }
    if (ret == 0) {
        for (int k = 0; k < N; ++k) { U_opt[k] = x[2 * k]; U_opt[N + k] = x[2 * k + 1]; }
        if (objective) {
            double o = qp.cst;
            mat_vec(qp.P, n, n, x, tmp);
            for (int j = 0; j < n; ++j) o += 0.5 * x[j] * tmp[j] + qp.q[j] * x[j];
            *objective = o;
        }
    }
    free(G); free(h); free(x); free(s); free(lam); free(rd); free(rp); free(Gx); free(dx); free(ds); free(dl);
    free(K); free(w); free(rhs); free(tmp);
    qp_free(&qp);
    return ret;
}

/* ---------------------------------------------------------- closed loop */

/* MPC/main.py:9-18 */
double orc_d_steady_state(const orc_params* p, double v) {
    double num = p->Cr0 + p->Cr2 * (v * v);
    double den = p->Cm1 - p->Cm2 * v;
    return num / den;
}

/* MPC/main.py:28-32 */
void orc_vref_ramp(int N, double Ts, double v0, double v_cruise, double tramp, double* v) {
    for (int k = 0; k <= N; ++k) {
        double t = (double)k * Ts;
        v[k] = v0 + (v_cruise - v0) * orc_clamp(t / tramp, 0.0, 1.0);
    }
}

void orc_path_eval(const orc_path* path, double x, double* y, double* dydx) {
    if (path->kind == 0) {
        const double* c = path->c;
        *y = c[0] + x * (c[1] + x * (c[2] + x * c[3]));
        *dydx = c[1] + x * (2.0 * c[2] + x * 3.0 * c[3]);
    } else if (path->kind == 1) {
        const double* c = path->c;
        double a = c[1] * x + c[2];
        *y = c[0] * sin(a) + c[3];
        *dydx = c[0] * c[1] * cos(a);
    } else {
        int nk = path->nk;
        const double* xk = path->xk;
        const double* cf = path->coef;
        if (x <= xk[0]) {
            double t = x - xk[0];
            *y = cf[0] + cf[1] * t;
            *dydx = cf[1];
            return;
        }
        if (x >= xk[nk - 1]) {
            const double* q = cf + 4 * (nk - 2);
            double h = xk[nk - 1] - xk[nk - 2];
            double yend = q[0] + h * (q[1] + h * (q[2] + h * q[3]));
            double send = q[1] + h * (2.0 * q[2] + h * 3.0 * q[3]);
            *y = yend + send * (x - xk[nk - 1]);
            *dydx = send;
            return;
        }
        int j = 0;
        while (j < nk - 2 && x >= xk[j + 1]) ++j;
        const double* q = cf + 4 * j;
        double t = x - xk[j];
        *y = q[0] + t * (q[1] + t * (q[2] + t * q[3]));
        *dydx = q[1] + t * (2.0 * q[2] + t * 3.0 * q[3]);
    }
}

/* MPC/main.py:51-68 */
void orc_ref_window(const orc_path* path, double x_start, int N, double Ts, const double* vref, double* out) {
    double xs = x_start;
    for (int k = 0; k <= N; ++k) {
        if (k > 0) xs = xs + vref[k - 1] * Ts;
        double y, dy;
        orc_path_eval(path, xs, &y, &dy);
        out[3 * k + 0] = xs;
        out[3 * k + 1] = y;
        out[3 * k + 2] = atan(dy);
    }
}

/* natural cubic spline (second derivative 0 at both ends): tridiagonal solve for M_j */
void orc_spline_natural(int nk, const double* xk, const double* yk, double* coef) {
    int n = nk;
    double* M = calloc(n, sizeof(double));
    if (n > 2) {
        int ni = n - 2;
        double *a = malloc(sizeof(double) * ni), *b = malloc(sizeof(double) * ni), *cc = malloc(sizeof(double) * ni),
               *d = malloc(sizeof(double) * ni);
        for (int i = 1; i <= ni; ++i) {
            double h0 = xk[i] - xk[i - 1], h1 = xk[i + 1] - xk[i];
            a[i - 1] = h0;
            b[i - 1] = 2.0 * (h0 + h1);
            cc[i - 1] = h1;
            d[i - 1] = 6.0 * ((yk[i + 1] - yk[i]) / h1 - (yk[i] - yk[i - 1]) / h0);
        }
        for (int i = 1; i < ni; ++i) {
            double wt = a[i] / b[i - 1];
            b[i] -= wt * cc[i - 1];
            d[i] -= wt * d[i - 1];
        }
        M[ni] = d[ni - 1] / b[ni - 1];
        for (int i = ni - 2; i >= 0; --i) M[i + 1] = (d[i] - cc[i] * M[i + 2]) / b[i];
        free(a); free(b); free(cc); free(d);
    }
    for (int j = 0; j < n - 1; ++j) {
        double h = xk[j + 1] - xk[j];
        coef[4 * j + 0] = yk[j];
        coef[4 * j + 1] = (yk[j + 1] - yk[j]) / h - h * (2.0 * M[j] + M[j + 1]) / 6.0;
        coef[4 * j + 2] = M[j] / 2.0;
        coef[4 * j + 3] = (M[j + 1] - M[j]) / (6.0 * h);
    }
    free(M);
}

/* MPC/main.py:85-101 */
void orc_closed_loop(const orc_params* p, const orc_mpc_cfg* c, const orc_path* path, const double x0[6],
                     const double u0[2], const double* vref, int T, double* traj_x, double* traj_u, int* status,
                     int* iters) {
    int N = c->N;
    double x[6], up[2], f[6], uc[2];
    double* pref = malloc(sizeof(double) * 3 * (N + 1));
    memcpy(x, x0, sizeof(x));
    memcpy(up, u0, sizeof(up));
    memcpy(traj_x, x, sizeof(x));
    orc_warm* warm = c->warm_start ? calloc(1, sizeof(orc_warm)) : NULL;
    for (int t = 0; t < T; ++t) {
        orc_ref_window(path, x[0], N, c->Ts, vref, pref);
        orc_info info;
        int st = orc_mpc_step_warm(p, c, x, up, pref, vref, uc, NULL, NULL, &info, warm);
        if (status) status[t] = st;
        if (iters) iters[t] = info.iters;
        orc_f_cont(p, x, uc, f);
        for (int i = 0; i < 6; ++i) x[i] = x[i] + c->Ts * f[i];
        memcpy(traj_x + 6 * (t + 1), x, sizeof(x));
        traj_u[2 * t] = uc[0];
        traj_u[2 * t + 1] = uc[1];
        up[0] = uc[0]; up[1] = uc[1];
    }
    free(warm);
    free(pref);
}

void orc_closed_loop_batch(const orc_params* p, const orc_mpc_cfg* c, const orc_path* paths, int B,
                           const double* x0, const double* u0, const double* vref, int T, double* traj_x,
                           double* traj_u, int* status, int* iters, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int b = 0; b < B; ++b)
        orc_closed_loop(p, c, paths + b, x0 + 6 * b, u0 + 2 * b, vref, T, traj_x + (size_t)6 * (T + 1) * b,
                        traj_u + (size_t)2 * T * b, status ? status + (size_t)T * b : NULL,
                        iters ? iters + (size_t)T * b : NULL);
}
