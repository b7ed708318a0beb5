/*
 * trajmpc.h -- C ABI of libtrajmpc.so, the MI355X (gfx950) batched MPC step.
 *
 * Drop-in boundary for the reference's hot path, DorianaG01/trajectory_generation
 * MPC/mpc_6stati.py.  The reference exposes plain Python functions (no FFI); every
 * entry point below is the batched, device-resident form of one of them, and the
 * Python module trajectory_generation_amd/mpc_6stati.py binds these symbols with
 * ctypes behind the reference's own signatures (INTEGRATION.md shows the binding).
 *
 *   reference (file:line)                      entry point here
 *   mpc_6stati.py:9-19    Params               traj_vehicle_params / traj_default_params
 *   mpc_6stati.py:25-53   tire_forces          traj_tire_forces_batch
 *   mpc_6stati.py:55-71   f_cont               traj_f_cont_batch
 *   mpc_6stati.py:73-97   numerical_jacobian   traj_numerical_jacobian_batch
 *   mpc_6stati.py:99-109  linearize_discretize traj_linearize_discretize_batch
 *   mpc_6stati.py:111-117 lateral_error        traj_lateral_error_batch
 *   mpc_6stati.py:120-143 mpc_step kwargs      traj_mpc_config / traj_default_config
 *   mpc_6stati.py:120-275 mpc_step             traj_mpc_step_batch (rollout, FD linearization,
 *                                              condensed QP, ADMM + polish, status, info)
 *   mpc_6stati.py:180-275 QP half only         traj_mpc_qp_batch (caller supplies A_k, B_k, g_k)
 *   MPC/main.py:51-68     ref_window_from_x... traj_ref_window_batch
 *   MPC/main.py:85-101    closed-loop loop     traj_closed_loop_step (window + mpc_step + plant)
 *
 * Conventions
 *   - All array pointers are DEVICE pointers (hipMalloc / torch.cuda memory), row-major, float64
 *     (the reference computes in numpy float64).  Shapes are given per argument.
 *   - `stream` is a hipStream_t (NULL = default stream).  Calls are asynchronous; they never
 *     copy to the host or synchronize, so they can be captured in a hipGraph.  Scratch memory is
 *     always the caller's `workspace` (sizes from traj_mpc_workspace_bytes, plus
 *     traj_mpc_sb_workspace_bytes for the state-bound solver); the library never allocates.
 *   - Return value: 0 on success, negative TRAJ_E_* on argument / launch errors.
 *   - Per-instance solver outcome is written to `status` (TRAJ_STATUS_*, same numbering as the
 *     CVXPY status strings listed below).  Like mpc_6stati.py:257-262, an instance whose status
 *     is not OPTIMAL / OPTIMAL_INACCURATE gets u_cmd = u_prev and NaN in X_opt / U_opt / objective.
 *   - Ownership: the caller owns every buffer.  The library holds no global state (except the
 *     diagnostics pointer of traj_debug_set_stamps).
 *   - Thread safety: reentrant; use one stream per host thread.
 */
#ifndef TRAJMPC_H
#define TRAJMPC_H

#ifdef __cplusplus
extern "C" {
#endif

#define TRAJMPC_ABI_VERSION 4   /* 2: traj_mpc_qp_batch takes a workspace; traj_mpc_sb_workspace_bytes;
                                  * 3: the step / QP entry points take horizons up to TRAJ_MAX_N_GENERAL;
                                  * 4: the closed loop takes state bounds and every N <= TRAJ_MAX_N_GENERAL (1024);
                                  *    traj_closed_loop_workspace_bytes */

/* error codes (return values) */
#define TRAJ_OK 0
#define TRAJ_E_ARG (-1)          /* bad argument (null pointer, B < 0, N out of range, ...) */
#define TRAJ_E_UNSUPPORTED (-2)  /* configuration this build does not implement */
#define TRAJ_E_LAUNCH (-3)       /* HIP launch failure */
#define TRAJ_E_HANDOFF (-4)      /* traj_closed_loop_check: a fused-run instance hand-off timed out */

/* per-instance status codes: CVXPY strings in brackets (mpc_6stati.py:257-262) */
#define TRAJ_STATUS_OPTIMAL 0                /* "optimal" */
#define TRAJ_STATUS_OPTIMAL_INACCURATE 1     /* "optimal_inaccurate" */
#define TRAJ_STATUS_USER_LIMIT 2             /* "user_limit" (OSQP max_iter reached) */
#define TRAJ_STATUS_INFEASIBLE 3             /* "infeasible" */
#define TRAJ_STATUS_INFEASIBLE_INACCURATE 4  /* "infeasible_inaccurate" */
#define TRAJ_STATUS_UNBOUNDED 5              /* "unbounded" */
#define TRAJ_STATUS_SOLVER_ERROR 6           /* "Solver Error: SolverError" (non-finite data, ...) */

/* mpc_6stati.py:9-19 (g is carried for layout parity; unused by the model, as in the reference) */
typedef struct {
    double Cm1, Cm2, Cr0, Cr2, Br, Cr, Dr, Bf, Cf, Df, m, Iz, lf, lr, g, maxAlpha, vx_zero;
} traj_vehicle_params;

/* mpc_step keyword arguments (mpc_6stati.py:120-143) + QP solver settings.  Solver defaults are
 * CVXPY's OSQP settings (eps_abs = eps_rel = 1e-5, max_iter = 10000, polish on). */
typedef struct {
    int N;                            /* horizon: 1 <= N <= TRAJ_MAX_N for every entry point; the step / QP
                                       * entry points also take TRAJ_MAX_N < N <= TRAJ_MAX_N_GENERAL (general
                                       * solver, caller-owned scratch: traj_mpc_sb_workspace_bytes) */
    double Ts;                        /* sampling time */
    double q_c, q_phi, q_vx;          /* :128-131 */
    double R[4], Rd[4];               /* :132-133, 2x2 row-major; the symmetric part is used */
    double u_lo[2], u_hi[2];          /* u_bounds  :135-136 */
    double du_lo[2], du_hi[2];        /* du_bounds :137-138 */
    int has_x_lo, has_x_hi;           /* x_lo / x_hi given (:139-140, :208-213); a side at -inf / inf
                                       * (|bound| >= 1e30) adds no rows.  With a finite bound the step
                                       * runs the general condensed-QP solver (dense state rows), and so
                                       * does the closed loop (one step per launch sequence, ABI 4) */
    double x_lo[6], x_hi[6];
    double eps_abs, eps_rel, eps_prim_inf, rho, sigma, alpha, delta;
    int max_iter, check_interval, scaling_iters, polish, polish_refine_iter, adaptive_rho;
    double adaptive_rho_tol;
    int polish_mode;                  /* 0: OSQP polish; 1: exact polish (KKT-certified optimum) */
    int polish_max_pass;
    double cert_tol;
    int polish_max_rounds;
    int warm_start;                   /* closed loop: start ADMM from the previous step's adapted rho
                                       * (mpc_6stati.py:256 requests warm_start=True) */
} traj_mpc_config;

/* Horizon tiers (mpc_step takes any N, mpc_6stati.py:125):
 *   N <= TRAJ_MAX_N (40)                 the register-resident hot kernels (mpc_solve.h): every entry point;
 *   N <= 20                              the one-wave register-resident kernels (mpc_solve.h);
 *   TRAJ_SPLIT_MIN_N <= N <= TRAJ_MAX_N_SPLIT  without state bounds: the row-split kernel (mpc_split.h: K^-1 in registers,
 *                                        each row split across a lane pair joined by v_permlane32_swap, 2 waves per
 *                                        SIMD; the QP entry point keeps the two-wave capacity-80 kernel up to TRAJ_MAX_N);
 *   TRAJ_MAX_N_SPLIT < N <= TRAJ_MAX_N_LONG  without state bounds: the long-horizon kernel (mpc_long.h: the hot kernels'
 *                                        algorithm with one thread per QP variable -- 256 threads, 512 past N = 128 --
 *                                        K^-1 in LDS up to N = 64 and in the caller's scratch beyond);
 *   otherwise (state bounds, or N > TRAJ_MAX_N_LONG up to TRAJ_MAX_N_GENERAL) the general condensed-QP solver
 *                                        (mpc_general.h, one 256-thread workgroup per instance, its Cholesky factor
 *                                        in the caller's scratch).
 * Past TRAJ_MAX_N the step and QP entry points take the scratch of traj_mpc_sb_workspace_bytes; the closed-loop entry
 * points (traj_closed_loop_step / _run) run TRAJ_MAX_N < N <= TRAJ_MAX_N_LONG on the long-horizon kernel, one step per
 * launch sequence (rollout, Jacobians, the closed-loop long-horizon solve with the window, warm rho and plant update),
 * with the same extra scratch after the workspace; with state bounds, or past TRAJ_MAX_N_LONG, they run the general
 * solver, one step per launch sequence, for every N up to TRAJ_MAX_N_GENERAL (traj_closed_loop_workspace_bytes sizes
 * the workspace of every case). */
#define TRAJ_MAX_N 40
#define TRAJ_MAX_N_SPLIT 64      /* TRAJ_SPLIT_MIN_N <= N <= this: the row-split kernel (mpc_split.h), K^-1 rows in
                                  * registers split across lane pairs */
#define TRAJ_SPLIT_MIN_N 21
#define TRAJ_MAX_N_LONG 256   /* 128 < N: the long-horizon kernel's 512-thread instance (round 6) */
#define TRAJ_MAX_N_GENERAL 1024

int traj_abi_version(void);
const char* traj_status_string(int status);
const char* traj_error_string(int err);

/* defaults: mpc_6stati.py:9-19 and the mpc_step defaults (:120-143) with horizon N and step Ts */
int traj_default_params(traj_vehicle_params* p);
int traj_default_config(traj_mpc_config* c, int N, double Ts);

/* ---- physics (mpc_6stati.py:25-117), B independent points ---- */
int traj_tire_forces_batch(const traj_vehicle_params* p, int B, const double* x /*[B,6]*/,
                           const double* u /*[B,2]*/, double* out /*[B,3] Fy_f, Fy_r, Frx*/, void* stream);
int traj_f_cont_batch(const traj_vehicle_params* p, int B, const double* x /*[B,6]*/, const double* u /*[B,2]*/,
                      double* xdot /*[B,6]*/, void* stream);
int traj_numerical_jacobian_batch(const traj_vehicle_params* p, int B, const double* x /*[B,6]*/,
                                  const double* u /*[B,2]*/, double eps_x, double eps_u, double* Jx /*[B,6,6]*/,
                                  double* Ju /*[B,6,2]*/, double* f /*[B,6]*/, void* stream);
int traj_linearize_discretize_batch(const traj_vehicle_params* p, int B, double Ts, const double* xbar /*[B,6]*/,
                                    const double* ubar /*[B,2]*/, double* Ad /*[B,6,6]*/, double* Bd /*[B,6,2]*/,
                                    double* g /*[B,6]*/, void* stream);
int traj_lateral_error_batch(int B, const double* X, const double* Y, const double* Xref, const double* Yref,
                             const double* phiref, double* out /*[B]*/, void* stream);

/* Device workspace the MPC step needs for B instances of horizon N: the linearization A_k, B_k, g_k
 * handed from the linearize kernels to the solve kernel (B * N * 54 doubles), the rollout record
 * (x_k, f_k) per stage (B * N * 12 doubles), then the closed-loop record of the previous step
 * (B * 4 doubles: rho, valid flag, ADMM iterations, mean iterations of the last fused run), the
 * closed-loop solve order (B ints, longest first) and the fused run's step queue (B + 2 ints).  Pass the same buffer to every traj_closed_loop_step of one run;
 * step t = 0 starts cold.  For TRAJ_SPLIT_MIN_N <= N <= TRAJ_MAX_N_SPLIT the size includes the row-split kernel's scratch.
 * The closed loop at TRAJ_MAX_N_SPLIT < N <= TRAJ_MAX_N_LONG needs traj_mpc_workspace_bytes(B, N) +
 * traj_mpc_sb_workspace_bytes(B, N) bytes (the long-horizon kernel's scratch after the workspace). */
size_t traj_mpc_workspace_bytes(int B, int N);
/* Scratch of the general solver, which runs with state bounds (x_lo / x_hi given with a finite side,
 * mpc_6stati.py:208-213), and of the long-horizon kernel (every horizon N > TRAJ_MAX_N): B * ~20.5k doubles at
 * N = 20 (N > TRAJ_MAX_N adds the Cholesky factor, 4 N^2 doubles; the long-horizon kernel uses at most 2 (2N + 6)^2).  traj_mpc_step_batch then needs traj_mpc_workspace_bytes(B, N) + this many
 * bytes; traj_mpc_qp_batch this many.  0 for B < 0 or N outside 1 .. TRAJ_MAX_N_GENERAL. */
size_t traj_mpc_sb_workspace_bytes(int B, int N);

/* ---- the MPC step (mpc_6stati.py:120-275) for B independent instances ----
 * x0 [B,6], u_prev [B,2], path_ref [B,N+1,3], vref [B,N+1]  (vref None / scalar is expanded by the
 * caller, :155-160).  Outputs: u_cmd [B,2], status [B]; optional (may be NULL): objective [B],
 * X_opt [B,6,N+1], U_opt [B,2,N], iters [B] (ADMM iterations), polished [B] (1 if polish accepted).
 * workspace: device buffer of at least traj_mpc_workspace_bytes(B, N) bytes (+ traj_mpc_sb_workspace_bytes(B, N)
 * with state bounds or N > TRAJ_MAX_N). */
int traj_mpc_step_batch(const traj_vehicle_params* p, const traj_mpc_config* c, int B, const double* x0,
                        const double* u_prev, const double* path_ref, const double* vref, double* u_cmd,
                        int* status, double* objective, double* X_opt, double* U_opt, int* iters, int* polished,
                        void* workspace, size_t workspace_bytes, void* stream);

/* QP half only (mpc_6stati.py:180-275) with the linearization supplied by the caller:
 * Ad [B,N,6,6], Bd [B,N,6,2], g [B,N,6].  Same outputs as traj_mpc_step_batch.  workspace: only with state
 * bounds or N > TRAJ_MAX_N (>= traj_mpc_sb_workspace_bytes(B, N) bytes), otherwise may be NULL. */
int traj_mpc_qp_batch(const traj_vehicle_params* p, const traj_mpc_config* c, int B, const double* x0,
                      const double* u_prev, const double* path_ref, const double* vref, const double* Ad,
                      const double* Bd, const double* g, double* u_cmd, int* status, double* objective,
                      double* X_opt, double* U_opt, int* iters, int* polished, void* workspace,
                      size_t workspace_bytes, void* stream);

/* ---- closed loop (MPC/main.py) ----
 * Reference path per trajectory (build-defined geometry): kind[b] = 0 cubic polynomial
 * y = c0 + c1 x + c2 x^2 + c3 x^3 (parabola, main.py:64-66), 1 sinusoid y = c0 sin(c1 x + c2) + c3
 * (MPC/README.md:73-76), 2 natural cubic spline through nk[b] knots xk[b,:] with piece coefficients
 * coef[b,j,0..3] (linear extrapolation outside the knots).  pc [B,4]; xk [B,KMAX]; coef [B,KMAX-1,4]. */
typedef struct {
    int kmax;                 /* knot capacity per trajectory (>= 2 if any kind 2 path) */
    const int* kind;          /* [B] */
    const double* pc;         /* [B,4] */
    const int* nk;            /* [B] (kind 2) */
    const double* xk;         /* [B,kmax] */
    const double* coef;       /* [B,kmax-1,4] */
} traj_paths;

/* main.py:51-68: window from x_start [B] with vref [B,N+1] -> path_ref [B,N+1,3] (phi* = atan(dy/dx)) */
int traj_ref_window_batch(const traj_paths* paths, int B, int N, double Ts, const double* x_start,
                          const double* vref, double* path_ref, void* stream);

/* Workspace bytes of the closed-loop entry points below for configuration c and B trajectories (every tier: the
 * register-resident and row-split kernels' traj_mpc_workspace_bytes, the long-horizon kernel's scratch after it, and
 * with state bounds the general solver's scratch plus the step's window and u_cmd); 0 for a configuration the closed
 * loop does not take. */
size_t traj_closed_loop_workspace_bytes(const traj_mpc_config* c, int B);

/* One closed-loop step of main.py:85-101 for B trajectories, in place (1 <= N <= TRAJ_MAX_N_GENERAL; with state
 * bounds x_lo / x_hi (mpc_6stati.py:208-213), or past TRAJ_MAX_N_LONG, on the general solver, each step a fresh
 * mpc_step call -- cold rho, as the reference's per-call loop -- bit-identical to traj_mpc_step_batch on the loop's
 * state):
 *   path_ref = window(x[:,0]); u_cmd = mpc_step(x, u_prev, path_ref, vref); x += Ts f_cont(x, u_cmd);
 *   u_prev = u_cmd.   x [B,6], u_prev [B,2] are updated; vref [B,N+1].
 * If hist_x / hist_u are non-NULL the new state / command are also written to
 * hist_x[b, t+1, :] ([B,T+1,6]) and hist_u[b, t, :] ([B,T,2]) with T = hist_T.
 * status / iters [B] (optional) receive this step's solver outcome. */
int traj_closed_loop_step(const traj_vehicle_params* p, const traj_mpc_config* c, const traj_paths* paths, int B,
                          double* x, double* u_prev, const double* vref, int t, int hist_T, double* hist_x,
                          double* hist_u, int* status, int* iters, void* workspace, size_t workspace_bytes,
                          void* stream);

/* The same closed loop for `steps` consecutive steps t0 .. t0+steps-1 in ONE launch (the fused
 * form): every instance runs its own steps back to back in one workgroup, with the linearization
 * (rollout + Jacobians) inside the workgroup and the state, u_prev and warm-start rho kept on chip,
 * so no instance waits for the slowest instance of a step.  Results are bit-identical to `steps`
 * calls of traj_closed_loop_step.  status / iters (optional) are [steps, B]; hist_x / hist_u as
 * above with t0 + steps <= hist_T; x / u_prev hold the final state. */
int traj_closed_loop_run(const traj_vehicle_params* p, const traj_mpc_config* c, const traj_paths* paths, int B,
                         double* x, double* u_prev, const double* vref, int t0, int steps, int hist_T,
                         double* hist_x, double* hist_u, int* status, int* iters, void* workspace,
                         size_t workspace_bytes, void* stream);

/* Synchronizes `stream` and reports whether the last traj_closed_loop_run on this workspace lost an
 * instance hand-off: a workgroup that waited for an instance's previous step longer than the spin
 * bound (traj_debug_spin_limit) went on with the state it found, so the run's x / u_prev / history
 * are not the closed loop's -- TRAJ_E_HANDOFF, never TRAJ_OK, in that case.  Call it after every
 * traj_closed_loop_run (the Python wrapper batch.closed_loop_run does) and before the next run on the
 * same workspace (a run clears the flag when it starts). */
int traj_closed_loop_check(const void* workspace, size_t workspace_bytes, int B, int N, void* stream);

/* ---- dataset files (host memory) ----
 * traj_dataset_write_csv: the reference's CSV schema (generation_type1.py:139-158), written with nthreads
 * threads.  X [B,T+1,6] states, U [B,T,2] controls, noise [B,T+1,6] measurement noise (noisy file only),
 * ids [B] trajectory ids; row r of trajectory b has t = r * Ts, the last row's d / delta empty (NaN).
 * Either path may be NULL.  Floats are written as pandas' to_csv writes float64 (shortest round-trip
 * repr), so the files are byte-identical to the pandas writer's.  Replaces the per-trajectory
 * DataFrame concat + to_csv of generation_type1.py:295-339. */
int traj_dataset_write_csv(const char* clean_path, const char* noisy_path, int B, int T, double Ts,
                           const double* X, const double* U, const double* noise, const long long* ids,
                           int nthreads);
/* Data rows (header excluded) and columns of a CSV file; negative TRAJ_E_* on error. */
long long traj_dataset_csv_rows(const char* path, int* ncols);
/* All fields of the data rows as float64, row-major [rows, ncols] into out (e.g. pinned host memory);
 * empty fields are NaN.  The parse of data_loader.py:5-53's pd.read_csv, in nthreads threads. */
int traj_dataset_read_csv(const char* path, long long rows, int ncols, double* out, int nthreads);

/* ---- diagnostics ----
 * Subsequent MPC launches write, per instance b, 32 int64 slots at buf[32 b ..] (device memory):
 * [0..7] s_memtime at phase boundaries (start, inputs, rollout, linearization, condensing,
 * scaling, solver end, outputs), [8] KKT factorizations, [9] ADMM iterations, [10] polish passes,
 * [11] cycles in residual checks, [12] cycles in factorizations, [13] cycles in polish, [14] checks,
 * [16..19] s_memtime inside the condensing phase (staging issued, staging landed, stage loop, P rows).
 * NULL disables.  For profiling only; never enabled by the product path. */
int traj_debug_set_stamps(long long* buf);
/* Subsequent traj_closed_loop_run launches write, per work item q = step * B + rank, 4 int64 at
 * buf[4 q ..] (device memory, [steps * B, 4]): drawn from the queue, previous step seen (wait over),
 * step done (s_memrealtime, 100 MHz), workgroup.  NULL disables.  Diagnostics only. */
int traj_debug_set_item_stamps(long long* buf);

/* Per-kernel timing of the next max_steps traj_closed_loop_step calls: HIP events recorded on the
 * launch stream around rollout_kernel, jac_kernel, order_kernel and solve_kernel (0 frees them).
 * traj_debug_kernel_times synchronizes, returns the mean milliseconds per step of the four kernels
 * in ms[4] and the number of timed steps, and restarts the count.  For bench.py's roofline leg. */
int traj_debug_kernel_timing(int max_steps);
/* traj_closed_loop_run's grid: the resident workgroup slots of the device (0, default) or the given
 * count (at least ceil(B / 8)); each workgroup runs its instances step by step.  For tests. */
int traj_debug_fused_grid(int workgroups);
/* Polls of an instance's step counter before a fused-run hand-off is declared lost (0: the default,
 * 2^22 polls with s_sleep back-off, seconds).  For the test that the loss is reported. */
int traj_debug_spin_limit(int polls);
/* Fused-run queue order: the heaviest per_mille / 1000 of the instances (by the previous launch's mean
 * ADMM iterations) run `steps` steps ahead of the level front (default 1 step, 100 per mille; 0 = plain
 * level order).  Results do not depend on it.  For experiments and tests. */
int traj_debug_queue_lead(int steps, int per_mille);
/* Fused-run run-ahead: a workgroup that completes an instance's step takes that instance's next step itself (no
 * hand-off, no queue draw) while the step is at most `levels` levels past the queue's draw front (default 0 =
 * every item from the queue in its order: measured not better across workloads).  Each item is claimed once (per-instance claim counter in the
 * workspace).  Results do not depend on it.  For experiments and tests. */
int traj_debug_run_ahead(int levels);
/* Fused-run kernel instance, by waves per SIMD: 0 (default) = by capacity and launch length (capacity 40: 2, or
 * 3 from 200 steps on; capacity 80: 1); 1, 2 or 3 = forced where built (capacity 40: 2 and 3; capacity 80: 2 runs
 * the lean two-wave instance, 1 and 3 the default one-wave-per-SIMD instance; other capacities: the default).
 * Results do not depend on it (the instances are bit-identical).  For experiments and tests. */
int traj_debug_fused_waves(int waves);
int traj_debug_kernel_times(double* ms, int* n_steps);
/* traj_mpc_step_batch's linearization: 1 (default) inside the solve launch (one launch per call), 0 = the
 * rollout and Jacobian kernels before it.  Results do not depend on it (bit-identical).  For tests. */
int traj_debug_step_linearize(int in_kernel);
/* Horizons TRAJ_MAX_N < N <= n_max run the row-split kernel (default TRAJ_MAX_N_SPLIT), the rest of the long tier the
 * long-horizon kernel (0: every N > TRAJ_MAX_N on the long-horizon kernel).  Both restate the same solver; for the
 * tests that compare them.  Diagnostics only. */
int traj_debug_split_max_n(int n_max);
/* Horizons n_min <= N <= TRAJ_MAX_N run the row-split kernel on the step and closed-loop paths (21 .. TRAJ_MAX_N + 1;
 * default TRAJ_SPLIT_MIN_N = 21; TRAJ_MAX_N + 1 = none, the capacity-80 kernel then runs 20 < N <= TRAJ_MAX_N).  For the
 * experiments and tests that compare the two.  Diagnostics only. */
int traj_debug_split_min_n(int n_min);

#ifdef __cplusplus
}
#endif
#endif
