/*
 * riccati_ipm.c -- CPU ORACLE (test infrastructure only; see traj_oracle.h).
 *
 * The QP of MPC/mpc_6stati.py:180-250 in the SPARSE form the reference hands to CVXPY/OSQP:
 * decision variables X (6, N+1) and U (2, N), the dynamics X_{k+1} = A_k X_k + B_k U_k + g_k kept as
 * equality constraints (:185-193), box and rate rows (:195-213), cost :223-250.  Solved by a
 * primal-dual interior-point method (Mehrotra predictor-corrector) whose Newton systems are
 * factorized by a Riccati recursion over the stages -- the structure-exploiting factorization of the
 * sparse KKT matrix.  Unlike the condensed form (traj_oracle.c build_qp), nothing here propagates the
 * open-loop free response x_{k+1} = A_k x_k + g_k over the horizon: the recursions run through the
 * feedback (closed-loop) dynamics, so an unstable A_k (rho(A_k) up to 6.45 at Ts = 0.05, SURVEY.md
 * App. D) cannot overflow the problem data.  The optimum is the unique optimum of the reference's QP
 * (strictly convex in U), the point OSQP returns when it converges.
 *
 * Formulation (DESIGN.md "Structured IPM"):
 *   stage state s_k = (x_k, w_k), w_k = u_{k-1} (w_0 = u_prev is data), input u_k;
 *   s_{k+1} = [A_k 0; 0 0] s_k + [B_k; I] u_k + [g_k; 0];
 *   8 one-sided rows per stage (G z <= h): u_k <= u_hi, -u_k <= -u_lo, u_k - u_{k-1} <= du_hi,
 *   -(u_k - u_{k-1}) <= -du_lo (u_{-1} = u_prev; rows with an infinite bound are dropped).
 * The GPU kernel (trajectory_generation_amd/csrc/mpc_ipm.h) runs the same iteration in the same
 * operation order wherever that is cheap; its results are compared with these to a tolerance.
 */
#include "traj_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define IPM_INFTY 1e30
#define IPM_TAU 0.99   /* fraction to the boundary */

static double vmax_abs(const double* v, int n) {
    double m = 0.0;
    for (int i = 0; i < n; ++i) {
        double a = fabs(v[i]);
        if (a > m || a != a) m = a;
    }
    return m;
}

/* row i (0..7) of stage k: coefficient on u_k[a] and on u_{k-1}[a] (a = i & 1), bound h */
static void row_def(const orc_mpc_cfg* c, const double* u_prev, int k, int i, double* cu, double* cw, double* h,
                    int* active) {
    const int a = i & 1;
    double hb;
    switch (i >> 1) {
        case 0: *cu = 1.0; *cw = 0.0; hb = c->u_hi[a]; *active = hb < IPM_INFTY; break;
        case 1: *cu = -1.0; *cw = 0.0; hb = -c->u_lo[a]; *active = c->u_lo[a] > -IPM_INFTY; break;
        case 2: *cu = 1.0; *cw = -1.0; hb = c->du_hi[a]; *active = hb < IPM_INFTY; break;
        default: *cu = -1.0; *cw = 1.0; hb = -c->du_lo[a]; *active = c->du_lo[a] > -IPM_INFTY; break;
    }
    if (k == 0 && *cw != 0.0) {   /* u_{-1} = u_prev is data: the rate rows of stage 0 bound u_0 only */
        hb -= *cw * u_prev[a];
        *cw = 0.0;
    }
    *h = hb;
}

typedef struct {
    int N, m;
    const orc_mpc_cfg* c;
    const double *x0, *u_prev, *Q, *qv, *Ad, *Bd, *gd;
    double R2[4], D2[4];
    double *x, *u, *nu, *t, *lam, *h, *cu, *cw;
    int* act;
    double *re, *rg, *gx, *gu;
    double *P, *S, *Ri, *Pc, *p, *K, *kk;
    double *dx, *du, *nup, *dt, *dl, *e, *gam_u;
} ipm_t;

/* gradient of the cost at (x, u): gx_k = Q_k x_k + q_k (k = 1..N), gu_k (input and rate terms) */
static void cost_grad(ipm_t* w) {
    const int N = w->N;
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < 6; ++i) {
            double s = w->qv[6 * k + i];
            for (int j = 0; j < 6; ++j) s += w->Q[36 * k + 6 * i + j] * w->x[6 * k + j];
            w->gx[6 * k + i] = s;
        }
    for (int k = 0; k < N; ++k) {
        const double* uk = w->u + 2 * k;
        const double* um = k ? w->u + 2 * (k - 1) : w->u_prev;
        for (int a = 0; a < 2; ++a) {
            double s = w->R2[2 * a] * uk[0] + w->R2[2 * a + 1] * uk[1];
            s += w->D2[2 * a] * (uk[0] - um[0]) + w->D2[2 * a + 1] * (uk[1] - um[1]);
            if (k + 1 < N) {
                const double* up = w->u + 2 * (k + 1);
                s -= w->D2[2 * a] * (up[0] - uk[0]) + w->D2[2 * a + 1] * (up[1] - uk[1]);
            }
            w->gu[2 * k + a] = s;
        }
    }
}

/* (G' v) on u_k[a] */
static double gt_u(const ipm_t* w, const double* v, int k, int a) {
    double s = 0.0;
    for (int i = a; i < 8; i += 2) s += w->cu[8 * k + i] * v[8 * k + i];
    if (k + 1 < w->N)
        for (int i = a; i < 8; i += 2) s += w->cw[8 * (k + 1) + i] * v[8 * (k + 1) + i];
    return s;
}

/* (G u)_r */
static double g_row(const ipm_t* w, const double* u, int r) {
    const int k = r >> 3, a = r & 1;
    double s = w->cu[r] * u[2 * k + a];
    if (k > 0) s += w->cw[r] * u[2 * (k - 1) + a];
    return s;
}

/* residuals at the iterate: dynamics (pr_e), inequality rows (pr_g), stationarity (dr), gradient
 * scale (sd) */
static void residuals(ipm_t* w, double* pr_e, double* pr_g, double* dr, double* sd) {
    const int N = w->N;
    cost_grad(w);
    double me = 0.0, mg = 0.0, md = 0.0, sg = 0.0;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < 6; ++i) {
            double s = w->gd[6 * k + i] - w->x[6 * (k + 1) + i];
            for (int j = 0; j < 6; ++j) s += w->Ad[36 * k + 6 * i + j] * w->x[6 * k + j];
            s += w->Bd[12 * k + 2 * i] * w->u[2 * k] + w->Bd[12 * k + 2 * i + 1] * w->u[2 * k + 1];
            w->re[6 * k + i] = s;
            if (fabs(s) > me || s != s) me = fabs(s);
        }
    for (int r = 0; r < w->m; ++r) {
        w->rg[r] = w->act[r] ? g_row(w, w->u, r) + w->t[r] - w->h[r] : 0.0;
        if (fabs(w->rg[r]) > mg || w->rg[r] != w->rg[r]) mg = fabs(w->rg[r]);
    }
    /* stationarity: x rows Q_k x_k + q_k - nu_k + A_k' nu_{k+1}; u rows gu + G'lam + B_k' nu_{k+1}
     * (nu_{k+1} = multiplier of the dynamics of stage k, stored at nu[6k]) */
    for (int k = 1; k <= N; ++k)
        for (int i = 0; i < 6; ++i) {
            double s = w->gx[6 * k + i] - w->nu[6 * (k - 1) + i];
            if (k < N)
                for (int j = 0; j < 6; ++j) s += w->Ad[36 * k + 6 * j + i] * w->nu[6 * k + j];
            if (fabs(s) > md || s != s) md = fabs(s);
            if (fabs(w->gx[6 * k + i]) > sg) sg = fabs(w->gx[6 * k + i]);
        }
    for (int k = 0; k < N; ++k)
        for (int a = 0; a < 2; ++a) {
            double s = w->gu[2 * k + a] + gt_u(w, w->lam, k, a);
            for (int j = 0; j < 6; ++j) s += w->Bd[12 * k + 2 * j + a] * w->nu[6 * k + j];
            if (fabs(s) > md || s != s) md = fabs(s);
            if (fabs(w->gu[2 * k + a]) > sg) sg = fabs(w->gu[2 * k + a]);
        }
    *pr_e = me;
    *pr_g = mg;
    *dr = md;
    *sd = sg > 1.0 ? sg : 1.0;
}

/* Riccati factorization of the Newton system, matrices only: for k = N-1 .. 0
 *   Ruu = Huu_k + B^' P B^,  S = Hus_k + B^' P A^,  P_k = Qss_k + A^' P A^ - S' Ruu^-1 S,
 * P_N = [Q_N 0; 0 0] (P = P_{k+1}; A^, B^ the stage-state dynamics).  Stores P_k, S_k, Ruu_k^-1,
 * K_k = -Ruu^-1 S and Pc_k = P_{k+1} [r_e_k; 0].  Returns -1 when a Ruu is not positive definite. */
static int factor(ipm_t* w) {
    const int N = w->N;
    double* PN = w->P + 64 * N;
    memset(PN, 0, 64 * sizeof(double));
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) PN[8 * i + j] = w->Q[36 * N + 6 * i + j];
    for (int k = N - 1; k >= 0; --k) {
        const double* P = w->P + 64 * (k + 1);
        const double* A = w->Ad + 36 * k;
        const double* B = w->Bd + 12 * k;
        double W[8];
        for (int i = 0; i < 8; ++i) W[i] = w->act[8 * k + i] ? w->lam[8 * k + i] / w->t[8 * k + i] : 0.0;
        /* rate-row block M = 2 Rd_sym + diag(barrier), input block Huu = 2 R_sym + M + diag(barrier) */
        double M[4], Huu[4];
        for (int i = 0; i < 4; ++i) M[i] = w->D2[i];
        M[0] += W[4] + W[6];
        M[3] += W[5] + W[7];
        for (int i = 0; i < 4; ++i) Huu[i] = w->R2[i] + M[i];
        Huu[0] += W[0] + W[2];
        Huu[3] += W[1] + W[3];
        /* PA = Pxx A (6 x 6), BtP = B^' P (2 x 8) = B' P[0:6, :] + P[6:8, :] */
        double PA[36], BtP[16];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int l = 0; l < 6; ++l) s += P[8 * i + l] * A[6 * l + j];
                PA[6 * i + j] = s;
            }
        for (int a = 0; a < 2; ++a)
            for (int j = 0; j < 8; ++j) {
                double s = P[8 * (6 + a) + j];
                for (int l = 0; l < 6; ++l) s += B[2 * l + a] * P[8 * l + j];
                BtP[8 * a + j] = s;
            }
        /* Pc_k = P[:, 0:6] r_e_k */
        for (int i = 0; i < 8; ++i) {
            double s = 0.0;
            for (int l = 0; l < 6; ++l) s += P[8 * i + l] * w->re[6 * k + l];
            w->Pc[8 * k + i] = s;
        }
        /* S = [BtP[:, 0:6] A, -M] (2 x 8); Ruu = Huu + BtP B^ */
        double* S = w->S + 16 * k;
        for (int a = 0; a < 2; ++a) {
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int l = 0; l < 6; ++l) s += BtP[8 * a + l] * A[6 * l + j];
                S[8 * a + j] = s;
            }
            S[8 * a + 6] = -M[2 * a];
            S[8 * a + 7] = -M[2 * a + 1];
        }
        double Ruu[4];
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) {
                double s = BtP[8 * a + 6 + b];
                for (int l = 0; l < 6; ++l) s += BtP[8 * a + l] * B[2 * l + b];
                Ruu[2 * a + b] = Huu[2 * a + b] + s;
            }
        Ruu[1] = Ruu[2] = 0.5 * (Ruu[1] + Ruu[2]);
        const double det = Ruu[0] * Ruu[3] - Ruu[1] * Ruu[2];
        if (!(Ruu[0] > 0.0) || !(det > 0.0) || !isfinite(det)) return -1;
        double* Ri = w->Ri + 4 * k;
        Ri[0] = Ruu[3] / det;
        Ri[3] = Ruu[0] / det;
        Ri[1] = Ri[2] = -Ruu[1] / det;
        double* K = w->K + 16 * k;
        for (int a = 0; a < 2; ++a)
            for (int j = 0; j < 8; ++j) K[8 * a + j] = -(Ri[2 * a] * S[j] + Ri[2 * a + 1] * S[8 + j]);
        if (k == 0) break;
        /* P_k = [Q_k + A' Pxx A, 0; 0, M] + S' K, every entry (i, j) formed as (min, max) (symmetric) */
        double* Pk = w->P + 64 * k;
        for (int i = 0; i < 8; ++i)
            for (int j = i; j < 8; ++j) {
                double s = 0.0;
                if (i < 6 && j < 6) {
                    s = w->Q[36 * k + 6 * i + j];
                    for (int l = 0; l < 6; ++l) s += A[6 * l + i] * PA[6 * l + j];
                } else if (i >= 6 && j >= 6) {
                    s = M[2 * (i - 6) + (j - 6)];
                }
                s += S[i] * K[j] + S[8 + i] * K[8 + j];
                Pk[8 * i + j] = s;
                Pk[8 * j + i] = s;
            }
    }
    return 0;
}

/* Newton direction for the complementarity targets rc: linear Riccati pass + forward pass.
 * Fills dx (k = 1..N), du, nup (the new dynamics multipliers), dt, dl. */
static void solve_dir(ipm_t* w, const double* rc) {
    const int N = w->N;
    /* e_r = lam + (rc + lam r_g) / t; gamma_u = grad_u J + G' e (gamma_x = grad_x J) */
    for (int r = 0; r < w->m; ++r)
        w->e[r] = w->act[r] ? w->lam[r] + (rc[r] + w->lam[r] * w->rg[r]) / w->t[r] : 0.0;
    for (int k = 0; k < N; ++k)
        for (int a = 0; a < 2; ++a) w->gam_u[2 * k + a] = w->gu[2 * k + a] + gt_u(w, w->e, k, a);
    /* backward: p_N = [gamma_xN; 0]; v = P_{k+1} c_k + p_{k+1}; kk = -Ruu^-1 (gamma_u + B^' v);
     * p_k = [gamma_xk + A' v_x; 0] + S' kk */
    double* pN = w->p + 8 * N;
    for (int i = 0; i < 6; ++i) pN[i] = w->gx[6 * N + i];
    pN[6] = pN[7] = 0.0;
    for (int k = N - 1; k >= 0; --k) {
        const double* pk1 = w->p + 8 * (k + 1);
        const double* A = w->Ad + 36 * k;
        const double* B = w->Bd + 12 * k;
        double v[8];
        for (int i = 0; i < 8; ++i) v[i] = w->Pc[8 * k + i] + pk1[i];
        double g_u[2];
        for (int a = 0; a < 2; ++a) {
            double s = w->gam_u[2 * k + a] + v[6 + a];
            for (int l = 0; l < 6; ++l) s += B[2 * l + a] * v[l];
            g_u[a] = s;
        }
        const double* Ri = w->Ri + 4 * k;
        double* kk = w->kk + 2 * k;
        kk[0] = -(Ri[0] * g_u[0] + Ri[1] * g_u[1]);
        kk[1] = -(Ri[2] * g_u[0] + Ri[3] * g_u[1]);
        if (k == 0) break;
        const double* S = w->S + 16 * k;
        double* pk = w->p + 8 * k;
        for (int i = 0; i < 6; ++i) {
            double s = w->gx[6 * k + i];
            for (int l = 0; l < 6; ++l) s += A[6 * l + i] * v[l];
            pk[i] = s + S[i] * kk[0] + S[8 + i] * kk[1];
        }
        for (int i = 6; i < 8; ++i) pk[i] = S[i] * kk[0] + S[8 + i] * kk[1];
    }
    /* forward: ds_0 = 0; du_k = K_k ds_k + kk_k; ds_{k+1} = A^ ds_k + B^ du_k + [r_e_k; 0];
     * nu+_{k+1} = (P_{k+1} ds_{k+1} + p_{k+1})[0:6] */
    double ds[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < N; ++k) {
        const double* K = w->K + 16 * k;
        const double* A = w->Ad + 36 * k;
        const double* B = w->Bd + 12 * k;
        double du[2];
        for (int a = 0; a < 2; ++a) {
            double s = w->kk[2 * k + a];
            for (int j = 0; j < 8; ++j) s += K[8 * a + j] * ds[j];
            du[a] = s;
        }
        double dn[8];
        for (int i = 0; i < 6; ++i) {
            double s = w->re[6 * k + i] + B[2 * i] * du[0] + B[2 * i + 1] * du[1];
            for (int j = 0; j < 6; ++j) s += A[6 * i + j] * ds[j];
            dn[i] = s;
        }
        dn[6] = du[0];
        dn[7] = du[1];
        w->du[2 * k] = du[0];
        w->du[2 * k + 1] = du[1];
        const double* P = w->P + 64 * (k + 1);
        const double* p = w->p + 8 * (k + 1);
        for (int i = 0; i < 6; ++i) {
            w->dx[6 * (k + 1) + i] = dn[i];
            double s = p[i];
            for (int j = 0; j < 8; ++j) s += P[8 * i + j] * dn[j];
            w->nup[6 * k + i] = s;
        }
        memcpy(ds, dn, sizeof(ds));
    }
    /* dt = -r_g - G du ; dl = (rc - lam dt) / t */
    for (int r = 0; r < w->m; ++r) {
        if (!w->act[r]) { w->dt[r] = w->dl[r] = 0.0; continue; }
        w->dt[r] = -w->rg[r] - g_row(w, w->du, r);
        w->dl[r] = (rc[r] - w->lam[r] * w->dt[r]) / w->t[r];
    }
}

static double step_max(const ipm_t* w) {
    double a = 1.0;
    for (int r = 0; r < w->m; ++r) {
        if (!w->act[r]) continue;
        if (w->dt[r] < 0.0) { double s = -w->t[r] / w->dt[r]; if (s < a) a = s; }
        if (w->dl[r] < 0.0) { double s = -w->lam[r] / w->dl[r]; if (s < a) a = s; }
    }
    return a;
}

int orc_ipm_core(const orc_mpc_cfg* c, int N, const double* x0, const double* u_prev, const double* Q,
                 const double* qv, const double* Ad, const double* Bd, const double* gd, const double* xinit,
                 double* X, double* U, int* iters_out, double* res_out) {
    ipm_t w;
    memset(&w, 0, sizeof(w));
    w.N = N;
    w.m = 8 * N;
    w.c = c;
    w.x0 = x0; w.u_prev = u_prev; w.Q = Q; w.qv = qv; w.Ad = Ad; w.Bd = Bd; w.gd = gd;
    for (int i = 0; i < 4; ++i) {
        const int it = (i == 1) ? 2 : (i == 2) ? 1 : i;   /* transposed index: 2 x symmetric part */
        w.R2[i] = c->R[i] + c->R[it];
        w.D2[i] = c->Rd[i] + c->Rd[it];
    }
    const int m = w.m;
    w.x = calloc(6 * (N + 1), sizeof(double));
    w.gx = calloc(6 * (N + 1), sizeof(double));
    w.dx = calloc(6 * (N + 1), sizeof(double));
    w.nu = calloc(6 * N, sizeof(double));
    w.nup = calloc(6 * N, sizeof(double));
    w.re = calloc(6 * N, sizeof(double));
    w.u = calloc(2 * N, sizeof(double));
    w.gu = calloc(2 * N, sizeof(double));
    w.du = calloc(2 * N, sizeof(double));
    w.gam_u = calloc(2 * N, sizeof(double));
    double** vm[] = {&w.t, &w.lam, &w.h, &w.cu, &w.cw, &w.rg, &w.dt, &w.dl, &w.e};
    for (size_t i = 0; i < sizeof(vm) / sizeof(vm[0]); ++i) *vm[i] = calloc(m, sizeof(double));
    w.act = calloc(m, sizeof(int));
    w.P = calloc(64 * (N + 1), sizeof(double));
    w.p = calloc(8 * (N + 1), sizeof(double));
    w.S = calloc(16 * N, sizeof(double));
    w.K = calloc(16 * N, sizeof(double));
    w.Ri = calloc(4 * N, sizeof(double));
    w.Pc = calloc(8 * N, sizeof(double));
    w.kk = calloc(2 * N, sizeof(double));
    double* rc = calloc(m, sizeof(double));
    double* dta = calloc(m, sizeof(double));
    double* dla = calloc(m, sizeof(double));

    /* start: x = xinit (the nominal rollout, on which the linear model is exact for u = u_prev),
     * u = u_prev clipped to the box, nu = 0, t = max(h - G u, 1), lam = 1 */
    for (int i = 0; i < 6; ++i) w.x[i] = x0[i];
    if (xinit)
        for (int i = 6; i < 6 * (N + 1); ++i) w.x[i] = xinit[i];
    for (int k = 0; k < N; ++k)
        for (int a = 0; a < 2; ++a) {
            double v = u_prev[a];
            v = (v < c->u_lo[a]) ? c->u_lo[a] : v;
            v = (v > c->u_hi[a]) ? c->u_hi[a] : v;
            w.u[2 * k + a] = v;
        }
    int nact = 0;
    for (int r = 0; r < m; ++r) {
        row_def(c, u_prev, r >> 3, r & 7, &w.cu[r], &w.cw[r], &w.h[r], &w.act[r]);
        if (w.act[r]) {
            const double s = w.h[r] - g_row(&w, w.u, r);
            w.t[r] = s > 1.0 ? s : 1.0;
            w.lam[r] = 1.0;
            ++nact;
        }
    }
    const double nd = (double)(nact > 0 ? nact : 1);
    const double tol = c->ipm_tol, loose = c->eps_rel;
    int status = ORC_USER_LIMIT, it = 0;
    double pr_e = 0, pr_g = 0, dr = 0, sd = 1, mu = 0;
    for (;; ++it) {
        residuals(&w, &pr_e, &pr_g, &dr, &sd);
        mu = 0.0;
        for (int r = 0; r < m; ++r) mu += w.act[r] ? w.t[r] * w.lam[r] : 0.0;
        mu /= nd;
        double sp = vmax_abs(w.x, 6 * (N + 1));
        const double su = vmax_abs(w.u, 2 * N);
        sp = (su > sp || su != su) ? su : sp;
        sp = sp > 1.0 ? sp : 1.0;
        if (!isfinite(pr_e) || !isfinite(pr_g) || !isfinite(dr) || !isfinite(mu)) { status = ORC_SOLVER_ERROR; break; }
        /* converged: primal residuals and complementarity at tol; the stationarity residual at 1e3 tol
         * (it is a difference of terms of the gradient's size and stalls near 1e-13 of it) */
        const double td = 1e3 * tol;
        if (pr_e <= tol * sp && pr_g <= tol && dr <= td * sd && mu <= tol * sd) { status = ORC_OPTIMAL; break; }
        /* the best a stalled or exhausted iteration can still report */
        const int acceptable = pr_e <= td * sp && pr_g <= td && dr <= td * sd && mu <= td * sd;
        const int near = pr_e <= loose * sp && pr_g <= loose && dr <= loose * sd && mu <= loose * sd;
        if (it >= c->ipm_max_iter) {
            status = acceptable ? ORC_OPTIMAL : near ? ORC_OPTIMAL_INACCURATE : ORC_USER_LIMIT;
            break;
        }
        if (factor(&w) != 0) {
            /* the Newton system lost definiteness (barrier weights ~1/tol): keep the current iterate */
            status = acceptable ? ORC_OPTIMAL : near ? ORC_OPTIMAL_INACCURATE : ORC_SOLVER_ERROR;
            break;
        }
        /* predictor (affine) direction */
        for (int r = 0; r < m; ++r) rc[r] = w.act[r] ? -w.t[r] * w.lam[r] : 0.0;
        solve_dir(&w, rc);
        const double aa = step_max(&w);
        double mu_aff = 0.0;
        for (int r = 0; r < m; ++r)
            if (w.act[r]) mu_aff += (w.t[r] + aa * w.dt[r]) * (w.lam[r] + aa * w.dl[r]);
        mu_aff /= nd;
        const double ratio = mu > 0.0 ? mu_aff / mu : 0.0;
        const double sg = ratio * ratio * ratio;   /* Mehrotra's centering (mu_aff / mu)^3 */
        memcpy(dta, w.dt, sizeof(double) * m);
        memcpy(dla, w.dl, sizeof(double) * m);
        /* corrector direction (same factorization) */
        for (int r = 0; r < m; ++r) rc[r] = w.act[r] ? -w.t[r] * w.lam[r] + sg * mu - dta[r] * dla[r] : 0.0;
        solve_dir(&w, rc);
        double a = IPM_TAU * step_max(&w);
        if (a > 1.0) a = 1.0;
        for (int i = 6; i < 6 * (N + 1); ++i) w.x[i] += a * w.dx[i];
        for (int i = 0; i < 2 * N; ++i) w.u[i] += a * w.du[i];
        for (int i = 0; i < 6 * N; ++i) w.nu[i] += a * (w.nup[i] - w.nu[i]);
        for (int r = 0; r < m; ++r)
            if (w.act[r]) {
                w.t[r] += a * w.dt[r];
                w.lam[r] += a * w.dl[r];
            }
    }
    memcpy(X, w.x, sizeof(double) * 6 * (N + 1));
    memcpy(U, w.u, sizeof(double) * 2 * N);
    if (iters_out) *iters_out = it;
    if (res_out) {
        res_out[0] = pr_e; res_out[1] = pr_g; res_out[2] = dr; res_out[3] = mu; res_out[4] = sd;
    }
    free(w.x); free(w.gx); free(w.dx); free(w.nu); free(w.nup); free(w.re);
    free(w.u); free(w.gu); free(w.du); free(w.gam_u);
    for (size_t i = 0; i < sizeof(vm) / sizeof(vm[0]); ++i) free(*vm[i]);
    free(w.act); free(w.P); free(w.p); free(w.S); free(w.K); free(w.Ri); free(w.Pc); free(w.kk);
    free(rc); free(dta); free(dla);
    return status;
}

/* state cost of mpc_6stati.py:225-250 per stage as 1/2 x'Q_k x + q_k'x + const: rows
 * c0 = (sin phi*, -cos phi*, 0..) (lateral_error :111-117), c1 = e_phi, c2 = e_vx */
void orc_ipm_state_cost(const orc_mpc_cfg* c, const double* path_ref, const double* vref, double* Q, double* qv) {
    const int N = c->N;
    const double W[3] = {c->q_c, c->q_phi, c->q_vx};
    memset(Q, 0, sizeof(double) * 36 * (N + 1));
    memset(qv, 0, sizeof(double) * 6 * (N + 1));
    for (int k = 0; k <= N; ++k) {
        const double Xr = path_ref[3 * k], Yr = path_ref[3 * k + 1], Pr = path_ref[3 * k + 2];
        const double s = sin(Pr), co = cos(Pr);
        double* Qk = Q + 36 * k;
        double* qk = qv + 6 * k;
        const double cv[2] = {s, -co};
        const double t0 = s * Xr - co * Yr;
        for (int i = 0; i < 2; ++i) {
            for (int j = 0; j < 2; ++j) Qk[6 * i + j] += 2.0 * W[0] * cv[i] * cv[j];
            qk[i] += -2.0 * W[0] * cv[i] * t0;
        }
        Qk[6 * 2 + 2] += 2.0 * W[1];
        qk[2] += -2.0 * W[1] * Pr;
        Qk[6 * 3 + 3] += 2.0 * W[2];
        qk[3] += -2.0 * W[2] * vref[k];
    }
}
