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

}  // extern "C"
