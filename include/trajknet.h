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
