/*
 * trajknet.h -- C ABI of the KalmanNet inference ops in libtrajmpc.so (gfx950), float32.
 *
 * Reference: DorianaG01/trajectory_generation KalmanNet/kalman_net.py (KalmanNetNN) and
 * KalmanNet/vehicle_model.py (VehicleModel.f / .h, pt_f_cont, pt_tire_forces).  The Kalman-gain
 * network's dense layers run as library GEMMs (PyTorch-ROCm / hipBLASLt); everything around them is
 * fused here:
 *
 *   reference (file:line)                                  entry point here
 *   kalman_net.py:145-157 step_prior (denorm, f, h, renorm) traj_knet_prior_f32 (+ innovation y - m1y,
 *   vehicle_model.py:19-79,109-153 f (clamps, Euler), h     kalman_net.py:161-162)
 *   torch.nn.GRU cell (seq_len 1), gates r, z, n            traj_knet_gru_gates_f32
 *   kalman_net.py:169-178 KNet_step posterior update        traj_knet_update_f32
 *   kalman_net.py:145-216 whole step (throughput path)     traj_knet_front_f32 + traj_knet_fc2_f32 + traj_knet_back_f32
 *   test_prediction.py:67-112,198-221 sliding-window        traj_knet_rollout_eval_f32
 *     open-loop rollout + ADE / FDE
 *   (no reference counterpart) EKF baseline of config 5     traj_ekf_run_f64
 *
 * Conventions as trajmpc.h: device pointers, row-major, asynchronous on `stream`, 0 / TRAJ_E_*.
 */
#ifndef TRAJKNET_H
#define TRAJKNET_H

#include "trajmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* State clamp limits injected into the vehicle Params by the caller (vehicle_model.py:54-57,125-131),
 * in this order. */
typedef struct {
    float x_min, x_max, y_min, y_max, phi_min, phi_max, vx_min, vx_max, vy_min, vy_max, omega_min, omega_max;
} traj_knet_limits;

/* Prior of one KalmanNet step for B sequences (kalman_net.py:145-157 + :161-162):
 *   x_real  = x_post * x_std + x_mean                       (x_post: normalized posterior [B,6])
 *   u_real  = u * u_std + u_mean if u_mean/u_std else u     ([B,2])
 *   x_prior = clamp(x_real + Ts f(x_real, u_real))          (vehicle_model.py:109-134, clamped f)
 *   m1x_prior = (x_prior - x_mean) / x_std                  ([B,6])
 *   m1y       = (h(x_prior) - y_mean) / y_std               ([B,5], h = rows 0,1,3,4,5)
 *   dy        = y - m1y  if y != NULL                       ([B,5])
 * x_mean/x_std [6], y_mean/y_std [5], u_mean/u_std [2] (NULL: u is already real). */
int traj_knet_prior_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, int B,
                        const float* x_post, const float* u, const float* y, const float* x_mean,
                        const float* x_std, const float* y_mean, const float* y_std, const float* u_mean,
                        const float* u_std, float* m1x_prior, float* m1y, float* dy, void* stream);

/* PyTorch GRU cell update for B rows of hidden size H, gates in torch order (r, z, n):
 *   gi = x W_ih' + b_ih, gh = h W_hh' + b_hh  (both [B,3H], computed by the caller's GEMMs)
 *   r = sigmoid(gi_r + gh_r), z = sigmoid(gi_z + gh_z), n = tanh(gi_n + r * gh_n)
 *   h_out = (1 - z) * n + z * h                 (h, h_out [B,H]; h_out may alias h) */
int traj_knet_gru_gates_f32(int B, int H, const float* gi, const float* gh, const float* h, float* h_out,
                            void* stream);

/* Posterior (kalman_net.py:169-178): x_post = x_prior + sigmoid(innov_logit) * (KG @ dy),
 * KG [B,6,5] row-major (the reshape of FC2's output), dy [B,5], innov_logit: device scalar. */
int traj_knet_update_f32(int B, const float* x_prior, const float* KG, const float* dy, const float* innov_logit,
                         float* x_post, void* stream);

/* Fused step (throughput path): the weights of a KalmanNetNN (NNBuild with hidden_dim_gru = 128) as
 * device pointers, row-major like the state_dict (nn.Linear weight [out, in]; nn.GRU weight_ih_l0
 * [3H, in], weight_hh_l0 [3H, H], gates in torch order r, z, n). */
typedef struct {
    int m, n, hidden;              /* 6, 5, 128 */
    int d_fc5, d_fc1, d_fc7, d_fc3; /* FC5 / FC1 / FC7 / FC3 widths: m*in_mult, n*n, n, m*m (all <= 64) */
    const float *fc5_w, *fc5_b;                                    /* FC5.0 */
    const float *gru_q_wih, *gru_q_bih, *gru_q_whh, *gru_q_bhh;    /* GRU_Q */
    const float *gru_sigma_wih, *gru_sigma_bih, *gru_sigma_whh, *gru_sigma_bhh;   /* GRU_Sigma */
    const float *fc1_w, *fc1_b, *fc7_w, *fc7_b;                    /* FC1.0, FC7.0 */
    const float *gru_s_wih, *gru_s_bih, *gru_s_whh, *gru_s_bhh;    /* GRU_S */
    const float *fc3_w, *fc3_b, *fc4_w, *fc4_b;                    /* FC3.0, FC4.0 */
    const float* innov_logit;                                      /* scalar */
    int d_fc2h;                                                    /* FC2 hidden width 2H*out_mult (multiple of 256) */
    const float *fc2a_w, *fc2a_b, *fc2b_w, *fc2b_b;                /* FC2.0 [d_fc2h, 2H], FC2.2 [n*m, d_fc2h] */
} traj_knet_net;

/* The fused kernels read the eleven weight matrices from a packed copy made once per set of weights:
 * traj_knet_packed_bytes(net) bytes (0 for unsupported shapes), filled by traj_knet_pack_f32 on
 * `stream` (16-byte aligned buffer; layout P[k4][j][4] = W[j][4 k4 + c], zero past K).  Biases and
 * innov_logit are read through `net` itself, so its pointers must stay valid while the kernels run. */
size_t traj_knet_packed_bytes(const traj_knet_net* net);
int traj_knet_pack_f32(const traj_knet_net* net, float* packed, size_t bytes, void* stream);

/* One KNet_step (kalman_net.py:145-216, eval mode) is three launches, front -> fc2 -> back:
 *   front: prior (as traj_knet_prior_f32; u and y read with strides, e.g. column t of [B,2,T] /
 *          [B,5,T]), FC5, GRU_Q, GRU_Sigma, FC1, FC7, GRU_S; updates h_q, h_s [B,H] in place and writes
 *          x2 = [out_Sigma | h_S] [B,2H] (FC2's input), m1x_prior [B,m], dy [B,n];
 *   fc2:   FC2 (Linear -> ReLU -> Linear) on x2 as partial sums over blocks of 320 hidden units (256 when
 *          d_fc2h is not a multiple of 320) into the workspace ws (traj_knet_fc2_workspace_bytes(net, B) bytes), without materializing the
 *          [B, d_fc2h] hidden activation;
 *   back:  KG = FC2's output (bias + the partial sums in a fixed order; also written to KG_out [B, n*m]
 *          if not NULL), FC3 on cat(h_S, KG), FC4 on cat(out_Sigma, FC3) -> h_sigma [B,H] (the new
 *          h_Sigma), then x_post = m1x_prior + sigmoid(innov_logit) (KG dy); x_post is also written to
 *          out[b*out_stride_b + i*out_stride_c] if out != NULL.
 * TRAJ_E_UNSUPPORTED for shapes other than m=6, n=5, hidden=128 (FC5 / FC1+FC7 widths <= 32, FC3 <= 64,
 * d_fc2h a multiple of 256).  fc2a_w, fc2a_b and fc2b_w must be 16-byte aligned.  Results are deterministic (no atomics). */
int traj_knet_front_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, const traj_knet_net* net,
                        const float* packed, int B, const float* x_post, const float* u, int u_stride_b,
                        int u_stride_c, const float* y, int y_stride_b, int y_stride_c, const float* x_mean,
                        const float* x_std, const float* y_mean, const float* y_std, const float* u_mean,
                        const float* u_std, float* h_q, const float* h_sigma, float* h_s, float* m1x_prior, float* dy,
                        float* x2, void* stream);
size_t traj_knet_fc2_workspace_bytes(const traj_knet_net* net, int B);
int traj_knet_fc2_f32(const traj_knet_net* net, int B, const float* x2, float* ws, size_t ws_bytes, void* stream);
/* How traj_knet_fc2_f32 forms its products (process-wide; returns the previous mode, -1 for a bad mode):
 *   2 (default): every f32 operand as three bf16 terms (x = h + m + l exactly) on the bf16 matrix cores, six of
 *                the nine term products (the dropped ones are below 2^-23 |a b|), f32 accumulation;
 *   1:           the same terms and sums as 2 (bit-identical), every wave splitting the input tile itself;
 *   0:           the f32 matrix cores (each product exact, f32 accumulation).
 * All are float32-accurate sums in a summation order of their own, like any GEMM against the reference's. */
int traj_knet_set_fc2_mode(int mode);
int traj_knet_back_f32(const traj_knet_net* net, const float* packed, int B, const float* x2, const float* ws,
                       const float* m1x_prior, const float* dy, float* h_sigma, float* x_post, float* out,
                       int out_stride_b, int out_stride_c, float* KG_out, void* stream);

/* back(t) and front(t + 1) fused into one launch (the sequence runner's steady state: 2 launches per
 * step instead of 3).  Arguments as traj_knet_back_f32 (ws of step t, out column t; no KG_out) and
 * traj_knet_front_f32 (u, y of step t + 1); h_sigma, x_post, m1x_prior, dy and x2 are updated through
 * step t and then overwritten with step t + 1's values, h_q / h_s advanced to step t + 1.  Results are
 * bit-identical to the two separate launches. */
int traj_knet_back_front_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts,
                             const traj_knet_net* net, const float* packed, int B, const float* ws, float* out,
                             int out_stride_b, int out_stride_c, const float* u, int u_stride_b, int u_stride_c,
                             const float* y, int y_stride_b, int y_stride_c, const float* x_mean, const float* x_std,
                             const float* y_mean, const float* y_std, const float* u_mean, const float* u_std,
                             float* h_q, float* h_sigma, float* h_s, float* x_post, float* m1x_prior, float* dy,
                             float* x2, void* stream);

/* Sliding-window open-loop prediction scoring (test_prediction.py:198-221 with rollout_open_loop :67-87,
 * compute_metrics :89-103, get_error_profile :105-112), all windows of B sequences in one launch.
 * Window w of sequence b starts at t = t0 + w * step (w < nwin; test_prediction.py iterates
 * range(t0, T - H, step), whose length traj_knet_rollout_windows returns, -1 on bad arguments):
 *   x      = x_est[b*e_sb + c*e_sc + t*e_st] * x_std + x_mean   (the filter's normalized estimates, e.g.
 *            [B,6,T] with strides 6T, T, 1; x_mean = x_std = NULL: x_est is already real)
 *   x_k+1  = clamp(x_k + Ts f(x_k, u[b, :, t + k]))  (k < H; u [B,2,T] in real units, as the filter's f)
 *   e_k    = || x_k+1[X, Y] - x_gt[b, X:Y, t + 1 + k] ||   (x_gt [B,6,T] real)
 *   ade[b*nwin + w] = mean_k e_k, fde[...] = e_{H-1}; err_profile [B*nwin, H] is written when not NULL;
 *   pred [B*nwin, 6, H] receives the rolled-out states when not NULL.  x_gt = NULL: rollout only
 *   (rollout_open_loop; pred required, ade / fde / err_profile unused).
 * Requires t0 + (nwin - 1) * step + H <= T - 1 when scored, <= T for a bare rollout (TRAJ_E_ARG otherwise). */
int traj_knet_rollout_windows(int T, int H, int t0, int step);
int traj_knet_rollout_eval_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, int B, int T,
                               int H, int t0, int step, int nwin, const float* x_est, int e_sb, int e_sc, int e_st,
                               const float* x_mean, const float* x_std, const float* u, const float* x_gt, float* ade,
                               float* fde, float* err_profile, float* pred, void* stream);

/* Build-defined EKF baseline for config 5 ("MSE vs reference EKF"; the reference has no EKF, SURVEY.md
 * 8(f) f2), float64, one thread per sequence, all T steps in one launch:
 *   predict  x- = f(x+, u_t) (the clamped vehicle_model.py:109-134 step), F = df/dx by central
 *            differences (step 1e-6 max(1, |x_j|); clamped components give zero rows),
 *            P- = F P+ F' + diag(Q)
 *   update   H = rows 0,1,3,4,5; S = H P- H' + diag(R); K = P- H' S^-1 (Cholesky); x+ = x- + K (y_t - H x-);
 *            P+ = (I - K H) P- (I - K H)' + K diag(R) K'   (Joseph form)
 * y [B,5,T] measurements and u [B,2,T] controls in real units, x0 [B,6] initial estimate,
 * P0 / Q [6] and R [5] diagonals; x_est [B,6,T] receives x+ after each step. */
int traj_ekf_run_f64(const traj_vehicle_params* p, const traj_knet_limits* lim, double Ts, int B, int T,
                     const double* y, const double* u, const double* x0, const double* P0, const double* Q,
                     const double* R, double* x_est, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* TRAJKNET_H */
