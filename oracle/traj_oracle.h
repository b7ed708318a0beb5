/*
 * traj_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference hot path, used ONLY by tests/, by
 * __graft_entry__.smoke() as the checker, and by bench.py's cpu_baseline leg.
 * The product path (trajectory_generation_amd/, libtrajmpc.so) never links,
 * loads or calls anything in this directory.
 *
 * What it restates (reference = /root/reference, DorianaG01/trajectory_generation):
 *   MPC/mpc_6stati.py:9-19    Params                      -> orc_default_params
 *   MPC/mpc_6stati.py:21-23   clamp                       -> orc_clamp
 *   MPC/mpc_6stati.py:25-53   tire_forces                 -> orc_tire_forces
 *   MPC/mpc_6stati.py:55-71   f_cont                      -> orc_f_cont
 *   MPC/mpc_6stati.py:73-97   numerical_jacobian          -> orc_numerical_jacobian
 *   MPC/mpc_6stati.py:99-109  linearize_discretize        -> orc_linearize_discretize
 *   MPC/mpc_6stati.py:111-117 lateral_error               -> orc_lateral_error
 *   MPC/mpc_6stati.py:120-275 mpc_step (rollout, QP, solve, status, info)
 *                                                         -> orc_mpc_step / orc_mpc_step_batch
 *   MPC/main.py:9-18          d_steady_state              -> orc_d_steady_state
 *   MPC/main.py:28-32         vref_profile_ramp_cruise    -> orc_vref_ramp
 *   MPC/main.py:51-68         ref_window_from_x_with_vref -> orc_ref_window
 *   MPC/main.py:85-101        closed-loop simulation      -> orc_closed_loop
 *
 * The QP solver (the reference calls CVXPY -> OSQP, third-party, unpinned: see
 * README.md:70 / MPC/README.md:84, absent from this image) is restated from
 * OSQP 0.6's published algorithm (Stellato et al., "OSQP: an operator splitting
 * solver for quadratic programs", Math. Prog. Comp. 2020): Ruiz equilibration,
 * ADMM with sigma/alpha relaxation and adaptive rho, OSQP termination
 * criteria, and solution polishing, with CVXPY's OSQP defaults
 * (eps_abs = eps_rel = 1e-5, max_iter = 10000, polish = on).  The QP is solved
 * in condensed form (X eliminated through the equality constraints
 * mpc_6stati.py:187-193, which fix X uniquely given U); the optimum is unique
 * because the cost is strictly convex in U (R > 0).
 */
#ifndef TRAJ_ORACLE_H
#define TRAJ_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    double Cm1, Cm2, Cr0, Cr2, Br, Cr, Dr, Bf, Cf, Df, m, Iz, lf, lr, g, maxAlpha, vx_zero;
} orc_params;

typedef struct {
    int N;
    double Ts;
    double q_c, q_phi, q_vx;
    double R[4], Rd[4];             /* 2x2 row-major */
    double u_lo[2], u_hi[2], du_lo[2], du_hi[2];
    int has_x_lo, has_x_hi;
    double x_lo[6], x_hi[6];
    /* OSQP settings */
    double eps_abs, eps_rel, eps_prim_inf, rho, sigma, alpha, delta;
    int max_iter, check_interval, scaling_iters, polish, polish_refine_iter, adaptive_rho;
    double adaptive_rho_tol;
    /* polish_mode 0: OSQP polish (one reduced-KKT solve, accepted if residuals drop).
     * polish_mode 1: exact polish -- the same reduced-KKT solve iterated as a primal-dual
     * active-set method until the active set is stable and the KKT conditions (incl. multiplier
     * signs) hold to cert_tol; the result is then the exact optimum of the QP. */
    int polish_mode, polish_max_pass;
    double cert_tol;
    int polish_max_rounds;   /* exact mode: ADMM continuation rounds (tolerance x 1e-2 each) */
    int warm_start;          /* closed loop: start ADMM from the previous step's rho (orc_warm) */
    /* QP solver (include/trajmpc.h traj_mpc_config.solver): 0 auto -- the condensed ADMM for
     * N < ORC_IPM_AUTO_MIN_N, falling back to the structured IPM (riccati_ipm.c, sparse form) when it
     * fails numerically (non-finite condensed data, failed factorization, max_iter), the structured
     * IPM for longer horizons; 1 condensed ADMM only; 2 structured IPM only; 3 condensed ADMM + IPM
     * fallback at any N */
    int solver;
    int ipm_max_iter;
    double ipm_tol;          /* relative KKT residual the IPM stops at */
} orc_mpc_cfg;

#define ORC_IPM_AUTO_MIN_N 33

/* status codes (identical numbering to include/trajmpc.h) */
enum {
    ORC_OPTIMAL = 0, ORC_OPTIMAL_INACCURATE = 1, ORC_USER_LIMIT = 2, ORC_INFEASIBLE = 3,
    ORC_INFEASIBLE_INACCURATE = 4, ORC_UNBOUNDED = 5, ORC_SOLVER_ERROR = 6
};

typedef struct {
    int status;
    int iters;
    int polished;      /* 1 if polish succeeded */
    double prim_res, dual_res, rho_final;
    double objective;
} orc_info;

void orc_default_params(orc_params* p);
void orc_default_cfg(orc_mpc_cfg* c, int N, double Ts);

double orc_clamp(double x, double lo, double hi);
void orc_tire_forces(const orc_params* p, const double x[6], const double u[2], double out[3]);
/* Tire sine evaluation (mpc_6stati.py:46-47): 0 = libm sin (default; the reference fixtures pin it), 1 = the HIP
 * path's bounded-range polynomial (trajmpc physics.h tire_sin_poly, same coefficients and fma order).  Returns the
 * previous mode.  Process-global. */
int orc_set_tire_sine(int mode);
/* The tire sine in the current mode (for the test that bounds the polynomial against libm). */
double orc_tire_sin(double z);
void orc_f_cont(const orc_params* p, const double x[6], const double u[2], double xdot[6]);
void orc_numerical_jacobian(const orc_params* p, const double x[6], const double u[2],
                            double eps_x, double eps_u, double Jx[36], double Ju[12], double f[6]);
void orc_linearize_discretize(const orc_params* p, const double xbar[6], const double ubar[2], double Ts,
                              double Ad[36], double Bd[12], double g[6]);
double orc_lateral_error(double X, double Y, double Xref, double Yref, double phiref);

/* nominal rollout mpc_6stati.py:165-172: xbar (6, N+1) row-major */
void orc_nominal_rollout(const orc_params* p, const double x0[6], const double u_prev[2], int N, double Ts,
                         double* xbar);

/* One MPC step. path_ref (N+1,3) row-major, vref (N+1).
 * Outputs: u_cmd (2) (u_prev on failure, mpc_6stati.py:257-262), X_opt (6,N+1) row-major,
 * U_opt (2,N) row-major (may be NULL), info. Returns status. */
int orc_mpc_step(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                 const double* path_ref, const double* vref, double u_cmd[2], double* X_opt, double* U_opt,
                 orc_info* info);

/* Closed-loop warm start (not in the reference, whose cvxpy problem is rebuilt every call): ADMM
 * starts from the step-size rho the previous step's solve adapted to, instead of cfg->rho.  The
 * iterates still start at zero (shifting the previous primal/dual solution was measured to lengthen
 * the iteration tail), and the polished optimum does not depend on rho. */
typedef struct {
    int valid;
    double rho;
} orc_warm;

/* orc_mpc_step with an optional warm start (read if warm->valid, always written back). */
int orc_mpc_step_warm(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                      const double* path_ref, const double* vref, double u_cmd[2], double* X_opt, double* U_opt,
                      orc_info* info, orc_warm* warm);

/* Batched: x0 [B,6], u_prev [B,2], path_ref [B,N+1,3], vref [B,N+1]; u_cmd [B,2], status [B],
 * objective [B], X_opt [B,6,N+1], U_opt [B,2,N], iters [B] (optional pointers may be NULL).
 * nthreads <= 0 -> OpenMP default. */
void orc_mpc_step_batch(const orc_params* p, const orc_mpc_cfg* c, int B, const double* x0,
                        const double* u_prev, const double* path_ref, const double* vref, double* u_cmd,
                        int* status, double* objective, double* X_opt, double* U_opt, int* iters,
                        int* polished, int nthreads);
/* the same with a per-instance warm start: rho[b] / valid[b] in (an orc_warm) and out (the closed loop's carried rho) */
void orc_mpc_step_batch_warm(const orc_params* p, const orc_mpc_cfg* c, int B, const double* x0,
                             const double* u_prev, const double* path_ref, const double* vref, double* rho,
                             int* valid, double* u_cmd, int* status, int* iters, int* polished, int nthreads);

/* Exact QP solve used to validate the ADMM restatement (dense primal active-set on the condensed QP,
 * box+rate rows only).  Returns 0 on success. U_opt (2,N) row-major. */
int orc_qp_exact(const orc_params* p, const orc_mpc_cfg* c, const double x0[6], const double u_prev[2],
                 const double* path_ref, const double* vref, double* U_opt, double* objective);

/* ---- structured interior-point solve of the sparse-form QP (riccati_ipm.c) ----
 * Q [N+1,36] / qv [N+1,6]: state cost per stage (orc_ipm_state_cost); Ad/Bd/gd the linearization
 * ([N,36], [N,12], [N,6]); xinit [N+1,6] starting states or NULL.  Outputs X [N+1,6], U [N,2] (stage-
 * major), iterations, residuals (dynamics, rows, stationarity, mu, gradient scale).  Returns a status. */
int orc_ipm_core(const orc_mpc_cfg* c, int N, const double* x0, const double* u_prev, const double* Q,
                 const double* qv, const double* Ad, const double* Bd, const double* gd, const double* xinit,
                 double* X, double* U, int* iters, double* res);
void orc_ipm_state_cost(const orc_mpc_cfg* c, const double* path_ref, const double* vref, double* Q, double* qv);
/* The QP half (mpc_6stati.py:180-275) by the structured IPM with the linearization given (Ad [N,6,6],
 * Bd [N,6,2], gd [N,6]); U_opt (2,N), X_opt (6,N+1) row-major (may be NULL); info->polished = -1. */
int orc_qp_ipm(const orc_mpc_cfg* c, const double x0[6], const double u_prev[2], const double* path_ref,
               const double* vref, const double* Ad, const double* Bd, const double* gd, const double* xinit,
               double* U_opt, double* X_opt, orc_info* info);

/* ---- closed-loop caller (MPC/main.py) ---- */
double orc_d_steady_state(const orc_params* p, double v);
void orc_vref_ramp(int N, double Ts, double v0, double v_cruise, double tramp, double* v);

/* Reference path descriptor (build-defined; see DESIGN.md "reference paths").
 * kind 0: polynomial y = c[0] + c[1] x + c[2] x^2 + c[3] x^3   (parabola: main.py:64-66)
 * kind 1: sinusoid   y = c[0] sin(c[1] x + c[2]) + c[3]        (MPC/README.md:73-76)
 * kind 2: natural cubic spline, nk knots xk[], piece coefficients coef[4*(nk-1)]
 *         (a,b,c,d) per piece, y = a + b t + c t^2 + d t^3, t = x - xk[j];
 *         linear extrapolation outside [xk[0], xk[nk-1]]. */
typedef struct {
    int kind, nk;
    double c[4];
    const double* xk;
    const double* coef;
} orc_path;

void orc_path_eval(const orc_path* path, double x, double* y, double* dydx);
/* main.py:51-68 with the geometry replaced by `path` (phi* = atan(dy/dx)). out (N+1,3) row-major */
void orc_ref_window(const orc_path* path, double x_start, int N, double Ts, const double* vref, double* out);

/* Natural cubic spline coefficients through (xk, yk), nk >= 2 knots: coef[4*(nk-1)] */
void orc_spline_natural(int nk, const double* xk, const double* yk, double* coef);

/* main.py:85-101: T closed-loop steps.  traj_x (T+1,6) states, traj_u (T,2) commands, status (T).
 * vref is a fixed (N+1) profile re-used each step (main.py:87). */
void orc_closed_loop(const orc_params* p, const orc_mpc_cfg* c, const orc_path* path, const double x0[6],
                     const double u0[2], const double* vref, int T, double* traj_x, double* traj_u,
                     int* status, int* iters);

/* B independent closed loops (OpenMP over trajectories): paths[B], x0 [B,6], u0 [B,2], vref (N+1)
 * shared; traj_x [B,T+1,6], traj_u [B,T,2], status [B,T], iters [B,T] (status/iters may be NULL). */
void orc_closed_loop_batch(const orc_params* p, const orc_mpc_cfg* c, const orc_path* paths, int B,
                           const double* x0, const double* u0, const double* vref, int T, double* traj_x,
                           double* traj_u, int* status, int* iters, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
