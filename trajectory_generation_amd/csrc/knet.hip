// knet.hip -- fused KalmanNet step ops for gfx950 (float32, as the reference runs).
//
// Reference: KalmanNet/kalman_net.py:145-178 (step_prior, KNet_step) and KalmanNet/vehicle_model.py
// :19-79 (pt_tire_forces / pt_f_cont: the KNet physics variant -- vx_eff = max(|vx|, vx_zero) without
// sign, only alpha_f clamped, Frx on vx_eff, phi / vx / vy / omega pre-clamped), :109-134 (Euler step
// + clamp of all six states), :136-153 (h = rows 0,1,3,4,5).  Element-wise: one thread per sequence
// for the prior and the posterior, one per hidden unit for the GRU gates.  Constants are rounded to
// float32 as PyTorch rounds Python scalars against float32 tensors; transcendentals are the ROCm
// single-precision ones (last-ulp differences to the CPU reference).
#include <hip/hip_runtime.h>

#include "../../include/trajknet.h"

namespace {

__device__ __forceinline__ float clampf_(float x, float lo, float hi) {   // torch.clamp (NaN propagates)
    float t = (x < lo) ? lo : x;
    return (t > hi) ? hi : t;
}

struct KP {   // vehicle parameters rounded to float32
    float Cm1, Cm2, Cr0, Cr2, Br, Cr, Dr, Bf, Cf, Df, m, Iz, lf, lr, maxAlpha, vx_zero;
};

__global__ __launch_bounds__(256) void knet_prior_kernel(KP p, traj_knet_limits L, float Ts, int B,
                                                         const float* __restrict__ x_post, const float* __restrict__ u,
                                                         const float* __restrict__ y, const float* __restrict__ xm,
                                                         const float* __restrict__ xs, const float* __restrict__ ym,
                                                         const float* __restrict__ ys, const float* __restrict__ um,
                                                         const float* __restrict__ us, float* __restrict__ m1x_prior,
                                                         float* __restrict__ m1y, float* __restrict__ dy) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    float x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = __fadd_rn(__fmul_rn(x_post[6 * b + i], xs[i]), xm[i]);   // _denorm_x
    float d = u[2 * b], delta = u[2 * b + 1];
    if (um && us) {   // _denorm_u (only when u statistics were set)
        d = __fadd_rn(__fmul_rn(d, us[0]), um[0]);
        delta = __fadd_rn(__fmul_rn(delta, us[1]), um[1]);
    }
    // pt_f_cont (vehicle_model.py:45-79)
    const float phi = clampf_(x[2], L.phi_min, L.phi_max);
    const float vx = clampf_(x[3], L.vx_min, L.vx_max);
    const float vy = clampf_(x[4], L.vy_min, L.vy_max);
    const float om = clampf_(x[5], L.omega_min, L.omega_max);
    // pt_tire_forces (:19-42)
    const float avx = fabsf(vx);
    const float vx_eff = (avx > p.vx_zero || avx != avx) ? avx : p.vx_zero;   // torch.max(|vx|, 0.3)
    float alpha_f = __fadd_rn(-atan2f(__fadd_rn(__fmul_rn(om, p.lf), vy), vx_eff), delta);
    const float alpha_r = atan2f(__fsub_rn(__fmul_rn(om, p.lr), vy), vx_eff);
    alpha_f = clampf_(alpha_f, -p.maxAlpha, p.maxAlpha);
    const float Fy_f = __fmul_rn(p.Df, sinf(__fmul_rn(p.Cf, atanf(__fmul_rn(p.Bf, alpha_f)))));
    const float Fy_r = __fmul_rn(p.Dr, sinf(__fmul_rn(p.Cr, atanf(__fmul_rn(p.Br, alpha_r)))));
    const float Frx = __fsub_rn(__fsub_rn(__fmul_rn(__fsub_rn(p.Cm1, __fmul_rn(p.Cm2, vx_eff)), d), p.Cr0),
                                __fmul_rn(p.Cr2, __fmul_rn(vx_eff, vx_eff)));
    const float cphi = cosf(phi), sphi = sinf(phi), cdl = cosf(delta), sdl = sinf(delta);
    float xd[6];
    xd[0] = __fsub_rn(__fmul_rn(vx, cphi), __fmul_rn(vy, sphi));
    xd[1] = __fadd_rn(__fmul_rn(vx, sphi), __fmul_rn(vy, cphi));
    xd[2] = om;
    xd[3] = __fdiv_rn(__fadd_rn(__fsub_rn(Frx, __fmul_rn(Fy_f, sdl)), __fmul_rn(__fmul_rn(p.m, vy), om)), p.m);
    xd[4] = __fdiv_rn(__fsub_rn(__fadd_rn(Fy_r, __fmul_rn(Fy_f, cdl)), __fmul_rn(__fmul_rn(p.m, vx), om)), p.m);
    xd[5] = __fdiv_rn(__fsub_rn(__fmul_rn(__fmul_rn(Fy_f, p.lf), cdl), __fmul_rn(Fy_r, p.lr)), p.Iz);
    // f: Euler step + clamp of all states (:109-134)
    const float lo[6] = {L.x_min, L.y_min, L.phi_min, L.vx_min, L.vy_min, L.omega_min};
    const float hi[6] = {L.x_max, L.y_max, L.phi_max, L.vx_max, L.vy_max, L.omega_max};
    float xn[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) xn[i] = clampf_(__fadd_rn(x[i], __fmul_rn(Ts, xd[i])), lo[i], hi[i]);
    // renormalize; h = rows 0,1,3,4,5 (:136-153)
#pragma unroll
    for (int i = 0; i < 6; ++i) m1x_prior[6 * b + i] = __fdiv_rn(__fsub_rn(xn[i], xm[i]), xs[i]);
    const int hr[5] = {0, 1, 3, 4, 5};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float my = __fdiv_rn(__fsub_rn(xn[hr[j]], ym[j]), ys[j]);
        m1y[5 * b + j] = my;
        if (dy) dy[5 * b + j] = __fsub_rn(y[5 * b + j], my);
    }
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.0f / (1.0f + expf(-v)); }

__global__ __launch_bounds__(256) void knet_gru_kernel(int B, int H, const float* __restrict__ gi,
                                                       const float* __restrict__ gh, const float* h,
                                                       float* h_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * H) return;
    const int b = i / H, k = i - b * H;
    const float* gib = gi + (size_t)b * 3 * H;
    const float* ghb = gh + (size_t)b * 3 * H;
    // ATen GRUCell: r = sigmoid(h_r + i_r), z = sigmoid(h_z + i_z), n = tanh(i_n + h_n * r),
    // h' = (h - n) * z + n
    const float r = sigmoidf_(__fadd_rn(ghb[k], gib[k]));
    const float z = sigmoidf_(__fadd_rn(ghb[H + k], gib[H + k]));
    const float nn = tanhf(__fadd_rn(gib[2 * H + k], __fmul_rn(ghb[2 * H + k], r)));
    const float hv = h[i];
    h_out[i] = __fadd_rn(__fmul_rn(__fsub_rn(hv, nn), z), nn);
}

__global__ __launch_bounds__(256) void knet_update_kernel(int B, const float* __restrict__ xp,
                                                          const float* __restrict__ KG, const float* __restrict__ dy,
                                                          const float* __restrict__ logit, float* __restrict__ xo) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const float gamma = sigmoidf_(logit[0]);
    const float* K = KG + (size_t)b * 30;
    const float* e = dy + (size_t)b * 5;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        float s = 0.0f;
#pragma unroll
        for (int j = 0; j < 5; ++j) s = __fadd_rn(s, __fmul_rn(K[5 * i + j], e[j]));
        xo[6 * b + i] = __fadd_rn(xp[6 * b + i], __fmul_rn(gamma, s));
    }
}

// ---------------------------------------------------------------- EKF baseline (float64)
struct KPd {
    double Cm1, Cm2, Cr0, Cr2, Br, Cr, Dr, Bf, Cf, Df, m, Iz, lf, lr, maxAlpha, vx_zero;
    double lo[6], hi[6];
};

__device__ __forceinline__ double clampd_(double x, double lo, double hi) {
    double t = (x < lo) ? lo : x;
    return (t > hi) ? hi : t;
}

// vehicle_model.py:109-134 in float64: pre-clamped pt_f_cont, Euler step, clamp of all states
__device__ void veh_f(const KPd& p, double Ts, const double* x, double d, double delta, double* xn) {
    const double phi = clampd_(x[2], p.lo[2], p.hi[2]), vx = clampd_(x[3], p.lo[3], p.hi[3]);
    const double vy = clampd_(x[4], p.lo[4], p.hi[4]), om = clampd_(x[5], p.lo[5], p.hi[5]);
    const double avx = fabs(vx);
    const double vx_eff = (avx > p.vx_zero) ? avx : p.vx_zero;
    double af = -atan2(om * p.lf + vy, vx_eff) + delta;
    const double ar = atan2(om * p.lr - vy, vx_eff);
    af = clampd_(af, -p.maxAlpha, p.maxAlpha);
    const double Fyf = p.Df * sin(p.Cf * atan(p.Bf * af));
    const double Fyr = p.Dr * sin(p.Cr * atan(p.Br * ar));
    const double Frx = (p.Cm1 - p.Cm2 * vx_eff) * d - p.Cr0 - p.Cr2 * (vx_eff * vx_eff);
    double sphi, cphi, sd, cd;
    sincos(phi, &sphi, &cphi);
    sincos(delta, &sd, &cd);
    const double xd[6] = {vx * cphi - vy * sphi, vx * sphi + vy * cphi, om,
                          (Frx - Fyf * sd + p.m * vy * om) / p.m, (Fyr + Fyf * cd - p.m * vx * om) / p.m,
                          (Fyf * p.lf * cd - Fyr * p.lr) / p.Iz};
    for (int i = 0; i < 6; ++i) xn[i] = clampd_(x[i] + Ts * xd[i], p.lo[i], p.hi[i]);
}

__global__ __launch_bounds__(64) void ekf_kernel(KPd p, double Ts, int B, int T, const double* __restrict__ y,
                                                 const double* __restrict__ u, const double* __restrict__ x0,
                                                 const double* __restrict__ P0, const double* __restrict__ Q,
                                                 const double* __restrict__ R, double* __restrict__ xo) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int hr[5] = {0, 1, 3, 4, 5};
    double x[6], P[6][6];
    for (int i = 0; i < 6; ++i) {
        x[i] = x0[6 * b + i];
        for (int j = 0; j < 6; ++j) P[i][j] = (i == j) ? P0[i] : 0.0;
    }
    for (int t = 0; t < T; ++t) {
        const double d = u[((size_t)b * 2 + 0) * T + t], de = u[((size_t)b * 2 + 1) * T + t];
        // predict
        double xm[6], F[6][6];
        veh_f(p, Ts, x, d, de, xm);
        for (int j = 0; j < 6; ++j) {
            const double h = 1e-6 * fmax(1.0, fabs(x[j]));
            double xp[6], xq[6], fp[6], fq[6];
            for (int i = 0; i < 6; ++i) {
                xp[i] = x[i] + (i == j ? h : 0.0);
                xq[i] = x[i] - (i == j ? h : 0.0);
            }
            veh_f(p, Ts, xp, d, de, fp);
            veh_f(p, Ts, xq, d, de, fq);
            for (int i = 0; i < 6; ++i) F[i][j] = (fp[i] - fq[i]) / (2.0 * h);
        }
        double FP[6][6], Pm[6][6];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += F[i][k] * P[k][j];
                FP[i][j] = s;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += FP[i][k] * F[j][k];
                Pm[i][j] = s + (i == j ? Q[i] : 0.0);
            }
        // update: S = H Pm H' + R (5x5), Cholesky S = L L'
        double S[5][5], L[5][5] = {};
        for (int a = 0; a < 5; ++a)
            for (int c = 0; c < 5; ++c) S[a][c] = Pm[hr[a]][hr[c]] + (a == c ? R[a] : 0.0);
        for (int a = 0; a < 5; ++a) {
            for (int c = 0; c <= a; ++c) {
                double s = S[a][c];
                for (int k = 0; k < c; ++k) s -= L[a][k] * L[c][k];
                L[a][c] = (a == c) ? sqrt(s) : s / L[c][c];
            }
        }
        // K' = S^-1 (H Pm) : solve L L' K' = H Pm (columns of K' per state)
        double Kt[5][6];
        for (int j = 0; j < 6; ++j) {
            double z[5];
            for (int a = 0; a < 5; ++a) {
                double s = Pm[hr[a]][j];
                for (int k = 0; k < a; ++k) s -= L[a][k] * z[k];
                z[a] = s / L[a][a];
            }
            for (int a = 4; a >= 0; --a) {
                double s = z[a];
                for (int k = a + 1; k < 5; ++k) s -= L[k][a] * Kt[k][j];
                Kt[a][j] = s / L[a][a];
            }
        }
        double innov[5];
        for (int a = 0; a < 5; ++a) innov[a] = y[((size_t)b * 5 + a) * T + t] - xm[hr[a]];
        for (int i = 0; i < 6; ++i) {
            double s = 0.0;
            for (int a = 0; a < 5; ++a) s += Kt[a][i] * innov[a];
            x[i] = xm[i] + s;
        }
        // Joseph form: P = A Pm A' + K R K', A = I - K H
        double A[6][6];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double kh = 0.0;
                for (int a = 0; a < 5; ++a) kh += (hr[a] == j) ? Kt[a][i] : 0.0;
                A[i][j] = (i == j ? 1.0 : 0.0) - kh;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += A[i][k] * Pm[k][j];
                FP[i][j] = s;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double s = 0.0;
                for (int k = 0; k < 6; ++k) s += FP[i][k] * A[j][k];
                double kr = 0.0;
                for (int a = 0; a < 5; ++a) kr += Kt[a][i] * R[a] * Kt[a][j];
                P[i][j] = s + kr;
            }
        for (int i = 0; i < 6; ++i) xo[((size_t)b * 6 + i) * T + t] = x[i];
    }
}

inline int nblk(long long n, int t) { return (int)((n + t - 1) / t); }

}  // namespace

extern "C" {

int traj_knet_prior_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, int B,
                        const float* x_post, const float* u, const float* y, const float* x_mean,
                        const float* x_std, const float* y_mean, const float* y_std, const float* u_mean,
                        const float* u_std, float* m1x_prior, float* m1y, float* dy, void* stream) {
    if (!p || !lim || B < 0) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!x_post || !u || !x_mean || !x_std || !y_mean || !y_std || !m1x_prior || !m1y) return TRAJ_E_ARG;
    if (dy && !y) return TRAJ_E_ARG;
    KP k{(float)p->Cm1, (float)p->Cm2, (float)p->Cr0, (float)p->Cr2, (float)p->Br, (float)p->Cr, (float)p->Dr,
         (float)p->Bf,  (float)p->Cf,  (float)p->Df,  (float)p->m,   (float)p->Iz, (float)p->lf, (float)p->lr,
         (float)p->maxAlpha, (float)p->vx_zero};
    hipLaunchKernelGGL(knet_prior_kernel, dim3(nblk(B, 256)), dim3(256), 0, (hipStream_t)stream, k, *lim, Ts, B,
                       x_post, u, y, x_mean, x_std, y_mean, y_std, u_mean, u_std, m1x_prior, m1y, dy);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_knet_gru_gates_f32(int B, int H, const float* gi, const float* gh, const float* h, float* h_out,
                            void* stream) {
    if (B < 0 || H < 1) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!gi || !gh || !h || !h_out) return TRAJ_E_ARG;
    hipLaunchKernelGGL(knet_gru_kernel, dim3(nblk((long long)B * H, 256)), dim3(256), 0, (hipStream_t)stream, B, H,
                       gi, gh, h, h_out);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_knet_update_f32(int B, const float* x_prior, const float* KG, const float* dy, const float* innov_logit,
                         float* x_post, void* stream) {
    if (B < 0) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!x_prior || !KG || !dy || !innov_logit || !x_post) return TRAJ_E_ARG;
    hipLaunchKernelGGL(knet_update_kernel, dim3(nblk(B, 256)), dim3(256), 0, (hipStream_t)stream, B, x_prior, KG, dy,
                       innov_logit, x_post);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_ekf_run_f64(const traj_vehicle_params* p, const traj_knet_limits* lim, double Ts, int B, int T,
                     const double* y, const double* u, const double* x0, const double* P0, const double* Q,
                     const double* R, double* x_est, void* stream) {
    if (!p || !lim || B < 0 || T < 0) return TRAJ_E_ARG;
    if (B == 0 || T == 0) return TRAJ_OK;
    if (!y || !u || !x0 || !P0 || !Q || !R || !x_est) return TRAJ_E_ARG;
    KPd k{p->Cm1, p->Cm2, p->Cr0, p->Cr2, p->Br, p->Cr, p->Dr, p->Bf, p->Cf, p->Df, p->m, p->Iz, p->lf, p->lr,
          p->maxAlpha, p->vx_zero,
          {lim->x_min, lim->y_min, lim->phi_min, lim->vx_min, lim->vy_min, lim->omega_min},
          {lim->x_max, lim->y_max, lim->phi_max, lim->vx_max, lim->vy_max, lim->omega_max}};
    hipLaunchKernelGGL(ekf_kernel, dim3(nblk(B, 64)), dim3(64), 0, (hipStream_t)stream, k, Ts, B, T, y, u, x0, P0, Q,
                       R, x_est);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

}  // extern "C"
