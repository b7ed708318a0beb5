/* Sanitizer harness (test infrastructure, CPU only): drives the C oracle (oracle/traj_oracle.c, riccati_ipm.c)
 * through every entry point the tests use -- physics on random and non-finite points, the MPC step at several
 * horizons, polish modes, state bounds, degenerate inputs, the batched and closed-loop drivers, the exact and IPM
 * QP solvers -- built with -fsanitize=address,undefined by tests/test_sanitizers.py.  Any out-of-bounds access,
 * use-after-free, leak or undefined behaviour aborts with a report; the checksum is printed for the log only. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/traj_oracle.h"

static unsigned long long rs = 88172645463325252ull;
static double urand(double lo, double hi) {
    rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17;
    return lo + (hi - lo) * (double)(rs >> 11) * (1.0 / 9007199254740992.0);
}

static double acc = 0.0;
static void add(const double* v, int n) {
    for (int i = 0; i < n; ++i)
        if (isfinite(v[i])) acc += v[i];
}

static void window(double x0, int N, double Ts, const double* vref, double* pr) {
    double xs = x0;
    for (int k = 0; k <= N; ++k) {
        pr[3 * k] = xs;
        pr[3 * k + 1] = 0.1 * xs * xs;
        pr[3 * k + 2] = atan(0.2 * xs);
        xs += vref[k] * Ts;
    }
}

int main(void) {
    orc_params p;
    orc_default_params(&p);
    const double special[] = {0.0, -0.0, 1e-310, -1e-310, 1e300, -1e300, INFINITY, -INFINITY, NAN};
    /* physics */
    for (int i = 0; i < 3000; ++i) {
        double x[6], u[2], out[6], J[36], Ju[12], f[6], A[36], B[12], g[6];
        for (int j = 0; j < 6; ++j) x[j] = urand(-3, 3);
        for (int j = 0; j < 2; ++j) u[j] = urand(-1, 1);
        if (i % 7 == 0) x[i % 6] = special[i % 9];
        if (i % 11 == 0) u[i % 2] = special[(i / 11) % 9];
        orc_tire_forces(&p, x, u, out);
        add(out, 3);
        orc_f_cont(&p, x, u, out);
        add(out, 6);
        orc_numerical_jacobian(&p, x, u, 1e-5, 1e-5, J, Ju, f);
        add(J, 36);
        orc_linearize_discretize(&p, x, u, 0.05, A, B, g);
        add(A, 36);
        add(g, 6);
        { const double e = orc_lateral_error(x[0], x[1], x[2], x[3], x[4]); add(&e, 1); }
    }
    /* the MPC step: horizons, polish modes, state bounds, degenerate inputs */
    const int Ns[] = {1, 2, 8, 20, 33, 40, 41};
    for (int in = 0; in < 7; ++in)
        for (int mode = 0; mode < 2; ++mode)
            for (int sb = 0; sb < 2; ++sb) {
                const int N = Ns[in];
                const double Ts = (in & 1) ? 0.02 : 0.05;
                orc_mpc_cfg c;
                orc_default_cfg(&c, N, Ts);
                c.polish_mode = mode;
                c.solver = 1;
                if (sb) {
                    c.has_x_lo = c.has_x_hi = 1;
                    for (int j = 0; j < 6; ++j) { c.x_lo[j] = -INFINITY; c.x_hi[j] = INFINITY; }
                    c.x_lo[3] = 0.3; c.x_hi[3] = 1.6;
                }
                double* vref = malloc(sizeof(double) * (N + 1));
                double* pr = malloc(sizeof(double) * 3 * (N + 1));
                double* X = malloc(sizeof(double) * 6 * (N + 1));
                double* U = malloc(sizeof(double) * 2 * N);
                orc_vref_ramp(N, Ts, 0.8, 2.0, 2.0, vref);
                for (int rep = 0; rep < 4; ++rep) {
                    double x0[6] = {urand(-2, 2), urand(-2, 2), urand(-.3, .3), urand(.4, 1.5), urand(-.05, .05),
                                    urand(-1, 1)};
                    double up[2] = {urand(-.2, .5), urand(-.3, .3)}, uc[2];
                    if (rep == 1) up[0] = 3.0;                 /* infeasible rate chain */
                    if (rep == 2) x0[4] = NAN;                 /* non-finite state */
                    window(x0[0], N, Ts, vref, pr);
                    if (rep == 3) pr[3 * (N / 2) + 1] = INFINITY;   /* non-finite reference */
                    orc_info info;
                    memset(&info, 0, sizeof(info));
                    orc_mpc_step(&p, &c, x0, up, pr, vref, uc, X, U, &info);
                    add(uc, 2);
                    if (!sb && N <= 40 && rep == 0) {
                        double Uq[2 * 41], obj;
                        if (orc_qp_exact(&p, &c, x0, up, pr, vref, Uq, &obj) == 0) add(Uq, 2 * N);
                    }
                }
                free(vref); free(pr); free(X); free(U);
            }
    /* batched step (OpenMP) and the IPM QP half */
    {
        const int N = 20, Bn = 16;
        const double Ts = 0.05;
        orc_mpc_cfg c;
        orc_default_cfg(&c, N, Ts);
        c.solver = 1;
        double vref[21], x0[16 * 6], up[16 * 2], pr[16 * 21 * 3], uc[32], obj[16], X[16 * 6 * 21], U[16 * 40];
        int st[16], it[16], pol[16];
        orc_vref_ramp(N, Ts, 0.8, 2.0, 2.0, vref);
        double vr[16 * 21];
        for (int b = 0; b < Bn; ++b) {
            double xb[6] = {urand(-2, 2), urand(-2, 2), urand(-.3, .3), urand(.4, 1.5), urand(-.05, .05), urand(-1, 1)};
            memcpy(x0 + 6 * b, xb, sizeof(xb));
            up[2 * b] = urand(-.2, .5);
            up[2 * b + 1] = urand(-.3, .3);
            window(xb[0], N, Ts, vref, pr + 63 * b);
            memcpy(vr + 21 * b, vref, sizeof(vref));
        }
        orc_mpc_step_batch(&p, &c, Bn, x0, up, pr, vr, uc, st, obj, X, U, it, pol, 4);
        add(uc, 32);
        double A[20 * 36], Bm[20 * 12], g[20 * 6], xbar[6 * 21], Uo[40], Xo[6 * 21];
        orc_nominal_rollout(&p, x0, up, N, Ts, xbar);
        for (int k = 0; k < N; ++k) {
            double xk[6];
            for (int j = 0; j < 6; ++j) xk[j] = xbar[j * (N + 1) + k];
            orc_linearize_discretize(&p, xk, up, Ts, A + 36 * k, Bm + 12 * k, g + 6 * k);
        }
        orc_info info;
        orc_qp_ipm(&c, x0, up, pr, vr, A, Bm, g, NULL, Uo, Xo, &info);
        add(Uo, 40);
    }
    /* closed loop over the three path kinds (spline through orc_spline_natural) */
    {
        const int N = 12, Bn = 3, T = 15;
        const double Ts = 0.05;
        orc_mpc_cfg c;
        orc_default_cfg(&c, N, Ts);
        c.solver = 1;
        c.warm_start = 1;
        double xk[11], yk[11], coef[40], vref[13];
        for (int i = 0; i < 11; ++i) { xk[i] = -6 + 4 * i; yk[i] = urand(-1, 1); }
        orc_spline_natural(11, xk, yk, coef);
        orc_vref_ramp(N, Ts, 0.8, 2.0, 2.0, vref);
        orc_path paths[3];
        memset(paths, 0, sizeof(paths));
        paths[0].kind = 0; paths[0].c[2] = 0.1;
        paths[1].kind = 1; paths[1].c[0] = 0.5; paths[1].c[1] = 0.5; paths[1].c[2] = 0.3;
        paths[2].kind = 2; paths[2].nk = 11; paths[2].xk = xk; paths[2].coef = coef;
        double x0[18] = {0, .5, 0, 1, 0, 0, 1, 0, 0, .8, 0, 0, -1, .2, .1, 1.2, 0, .1}, u0[6] = {.1, 0, .1, 0, .1, 0};
        double tx[3 * 16 * 6], tu[3 * 15 * 2];
        int st[45], it[45];
        orc_closed_loop_batch(&p, &c, paths, Bn, x0, u0, vref, T, tx, tu, st, it, 3);
        add(tx, 3 * 16 * 6);
        double win[39];
        orc_ref_window(&paths[2], 50.0, N, Ts, vref, win);   /* extrapolation past the last knot */
        add(win, 39);
    }
    printf("san_oracle ok %.6g\n", acc);
    return 0;
}
