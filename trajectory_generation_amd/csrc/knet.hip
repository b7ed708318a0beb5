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

#include <atomic>

#include "../../include/trajknet.h"

namespace {

__device__ __forceinline__ float clampf_(float x, float lo, float hi) {   // torch.clamp (NaN propagates)
    float t = (x < lo) ? lo : x;
    return (t > hi) ? hi : t;
}

struct KP {   // vehicle parameters rounded to float32
    float Cm1, Cm2, Cr0, Cr2, Br, Cr, Dr, Bf, Cf, Df, m, Iz, lf, lr, maxAlpha, vx_zero;
};

// VehicleModel.f (vehicle_model.py:109-134) on one real state: xn = clamp(x + Ts f_cont(x, u))
__device__ __forceinline__ void veh_step(const KP& p, const traj_knet_limits& L, float Ts, const float* x, float d,
                                         float delta, float* xn) {
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
#pragma unroll
    for (int i = 0; i < 6; ++i) xn[i] = clampf_(__fadd_rn(x[i], __fmul_rn(Ts, xd[i])), lo[i], hi[i]);
}

// kalman_net.py:145-162 for one sequence: x_post (normalized) -> prior (normalized), m1y, dy = y - m1y
__device__ __forceinline__ void prior_one(const KP& p, const traj_knet_limits& L, float Ts, const float* xp, float d,
                                          float delta, const float* yv, int ystride, const float* xm,
                                          const float* xs, const float* ym, const float* ys, const float* um,
                                          const float* us, float* prior, float* m1y, float* dyo) {
    float x[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = __fadd_rn(__fmul_rn(xp[i], xs[i]), xm[i]);   // _denorm_x
    if (um && us) {   // _denorm_u (only when u statistics were set)
        d = __fadd_rn(__fmul_rn(d, us[0]), um[0]);
        delta = __fadd_rn(__fmul_rn(delta, us[1]), um[1]);
    }
    float xn[6];
    veh_step(p, L, Ts, x, d, delta, xn);
    // renormalize; h = rows 0,1,3,4,5 (:136-153)
#pragma unroll
    for (int i = 0; i < 6; ++i) prior[i] = __fdiv_rn(__fsub_rn(xn[i], xm[i]), xs[i]);
    const int hr[5] = {0, 1, 3, 4, 5};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float my = __fdiv_rn(__fsub_rn(xn[hr[j]], ym[j]), ys[j]);
        if (m1y) m1y[j] = my;
        if (dyo) dyo[j] = __fsub_rn(yv[j * ystride], my);
    }
}

__global__ __launch_bounds__(256) void knet_prior_kernel(KP p, traj_knet_limits L, float Ts, int B,
                                                         const float* __restrict__ x_post, const float* __restrict__ u,
                                                         const float* __restrict__ y, const float* __restrict__ xm,
                                                         const float* __restrict__ xs, const float* __restrict__ ym,
                                                         const float* __restrict__ ys, const float* __restrict__ um,
                                                         const float* __restrict__ us, float* __restrict__ m1x_prior,
                                                         float* __restrict__ m1y, float* __restrict__ dy) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    prior_one(p, L, Ts, x_post + 6 * b, u[2 * b], u[2 * b + 1], y ? y + 5 * b : nullptr, 1, xm, xs, ym, ys, um, us,
              m1x_prior + 6 * b, m1y + 5 * b, dy ? dy + 5 * b : nullptr);
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

// test_prediction.py:198-221 for every (sequence b, window w) at once: the window starts at
// t = t0 + w * step from the filter's estimate x_est[b, :, t] (normalized -> real, :202-203), runs
// rollout_open_loop (:67-87: H clamped Euler steps of f with u[b, :, t + k]) and scores the XY error
// against x_gt[b, :, t + 1 + k] (compute_metrics / get_error_profile, :89-112).  One thread per window;
// the serial chain is H steps of the same physics as the filter's prior (veh_step).
__global__ __launch_bounds__(64) void knet_rollout_kernel(KP p, traj_knet_limits L, float Ts, int B, int T, int H,
                                                          int t0, int step, int nwin, const float* __restrict__ xe,
                                                          int e_sb, int e_sc, int e_st,
                                                          const float* __restrict__ xm, const float* __restrict__ xs,
                                                          const float* __restrict__ u, const float* __restrict__ xg,
                                                          float* __restrict__ ade, float* __restrict__ fde,
                                                          float* __restrict__ prof, float* __restrict__ pred) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (i >= B * nwin) return;
    const int b = i / nwin, t = t0 + (i % nwin) * step;
    const float* eb = xe + (size_t)b * e_sb + (size_t)t * e_st;
    const float* ub = u + (size_t)b * 2 * T;
    const float* gb = xg ? xg + (size_t)b * 6 * T : nullptr;
    float x[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        const float v = eb[(size_t)c * e_sc];
        x[c] = xm ? __fadd_rn(__fmul_rn(v, xs[c]), xm[c]) : v;   // x_start_norm * x_std + x_mean
    }
    double sum = 0.0;
    float e = 0.0f;
    // each step's inputs are loaded one step ahead: a launch holds about one wave per SIMD (B * nwin
    // threads), so no other wave hides the load latency of the serial chain
    float ud = ub[t], ue = ub[T + t], gx = gb ? gb[t + 1] : 0.0f, gy = gb ? gb[T + t + 1] : 0.0f;
    for (int k = 0; k < H; ++k) {
        const float cd = ud, ce = ue, cgx = gx, cgy = gy;
        if (k + 1 < H) {
            ud = ub[t + k + 1];
            ue = ub[T + t + k + 1];
            if (gb) {
                gx = gb[t + k + 2];
                gy = gb[T + t + k + 2];
            }
        }
        float xn[6];
        veh_step(p, L, Ts, x, cd, ce, xn);
        if (gb) {
            const float dx = __fsub_rn(xn[0], cgx), dyv = __fsub_rn(xn[1], cgy);
            e = __fsqrt_rn(__fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dyv, dyv)));   // sqrt(sum(diff**2)) over X, Y
            sum += (double)e;
            if (prof) prof[(size_t)i * H + k] = e;
        }
        if (pred) {
#pragma unroll
            for (int c = 0; c < 6; ++c) pred[((size_t)i * 6 + c) * H + k] = xn[c];
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) x[c] = xn[c];
    }
    if (gb) {
        ade[i] = (float)(sum / (double)H);   // err_dist.mean()
        fde[i] = e;                          // err_dist[0, -1]
    }
}

// ---------------------------------------------------------------- fused step (throughput path)
// One KalmanNet step in two kernels around FC2 (kalman_net.py:145-216, eval mode):
//   front: prior -> FC5 -> GRU_Q -> GRU_Sigma -> FC1, FC7 -> GRU_S, writing x2 = [out_Sigma | h_S]
//          (FC2's input) and the hidden states;
//   back:  FC3 -> FC4 (the new h_Sigma) -> posterior update, from FC2's output KG.
// A workgroup owns KS sequences through every layer (no cross-workgroup dependency); activations stay
// in LDS, weights stream from L2 in the packed layout P[k4][j][4] = W[j][4 k4 + c] (zero past K), so
// the lanes of a wave (consecutive outputs j) read one contiguous 1 KiB run per float4 load.  GRU
// cells: a thread per hidden unit and K quarter forms the six gate dot products over its quarter; the
// thread (unit, quarter q) then adds the four quarters' partials of sequence q and applies torch's GRU
// gate math (as knet_gru_kernel).  Every dot product is a k-ordered fmaf chain
// started at the bias: float32 results within rounding of the library GEMM path.
constexpr int KS = 4;        // sequences per workgroup
constexpr int KH = 128;      // hidden size (hidden_dim_gru)
constexpr int KQ = 4;        // K parts of every dot product (thread t: unit t & 127, part t >> 7)
constexpr int KT = KH * KQ;  // threads per workgroup: 8 waves, two per SIMD

struct KNet {
    int m, n, dFC5, dFC1, dFC7, dFC3;
    const float *b5, *biQ, *bhQ, *biG, *bhG, *b1, *b7, *biS, *bhS, *b3, *b4, *logit, *b2b;
    const float4 *W5, *WiQ, *WhQ, *WiG, *WhG, *W1, *W7, *WiS, *WhS, *W3, *W4;   // packed
};

// packed rows of 4 k per matrix: K rounded up to a multiple of 64 (zero weights past K), so that each
// quarter of a split dot product runs a whole number of KD-row prefetch groups
__host__ __device__ inline int k4_(int K) { return ((K + 63) / 64) * 16; }

// Packed-buffer offsets (in floats) of the eleven matrices, in the order of traj_knet_net.
struct PackPlan {
    int N[11], K[11];
    size_t off[12];
};
static PackPlan pack_plan(const traj_knet_net* w) {
    PackPlan pl{};
    const int H = w->hidden;
    const int N[11] = {w->d_fc5, 3 * H, 3 * H, 3 * H, 3 * H, w->d_fc1, w->d_fc7, 3 * H, 3 * H, w->d_fc3, H};
    const int K[11] = {w->m, w->d_fc5, H, H, H, H, w->n, w->d_fc1 + w->d_fc7, H, H + w->n * w->m, H + w->d_fc3};
    pl.off[0] = 0;
    for (int i = 0; i < 11; ++i) {
        pl.N[i] = N[i];
        pl.K[i] = K[i];
        pl.off[i + 1] = pl.off[i] + (size_t)4 * k4_(K[i]) * N[i];
    }
    return pl;
}

__global__ void knet_pack_kernel(const float* __restrict__ W, int N, int K, float* __restrict__ P) {
    const int K4 = k4_(K);
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)K4 * N * 4) return;
    const int c = (int)(i & 3), j = (int)((i >> 2) % N), k4 = (int)((i >> 2) / N);
    const int k = 4 * k4 + c;
    P[i] = k < K ? W[(size_t)j * K + k] : 0.0f;
}

// Activations live in LDS k-major, xT[k][KS] (one float4 = the KS sequences' k-th input), rows
// zero-padded to a multiple of 4.  Dot products are split over K between the four quarters of the
// workgroup (thread t: output / hidden unit t & 127, K quarter t >> 7) and the quarters' partial sums
// are added through LDS in quarter order; weight loads run KD float4 rows ahead of the FMAs, and the
// two waves of each SIMD cover each other's L2 latency.
constexpr int KD = 4;   // (8 rows in flight for the GRU cells' 8-row quarters measured 71 vs 63 us per step, round 5)
#ifndef TRAJ_KNET_PK
#define TRAJ_KNET_PK 1   // dot_ks on explicit sequence-pair v_pk_fma_f32 (0: scalar fmaf chains, the compiler pairs them)
#endif

// acc[g][s] += sum_{k4 in [k4b, k4e)} xT[4 k4 + c][s] * P[k4][j + g * KH][c]  (P rows: NR per k4).
// Measured on MI355X (front launch, B = 1024): this compact runtime loop 24.7 us; the same loop with
// compile-time trip counts 27.5 us; fully unrolled straight-line code 29.4 us (register spills); a
// cross-layer chained prefetch gave nothing -- the chain is bound by per-layer barrier / LDS / load
// latency, not by one stalled group.
typedef float f2v __attribute__((ext_vector_type(2)));

template <int G>
__device__ __forceinline__ void dot_ks(const float* xT, int k4b, int k4e, const float4* __restrict__ P, int NR, int j,
                                       float (&acc)[G][KS]) {
#if TRAJ_KNET_PK
    // sequence pairs as packed f32 operands: v_pk_fma_f32 with the weight broadcast to both halves, the pairs straight
    // from the LDS float4s and the accumulators -- no register moves to assemble operand pairs (the same fmaf per
    // accumulator in the same k order as below, bit for bit)
    f2v a2[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        a2[g][0] = f2v{acc[g][0], acc[g][1]};
        a2[g][1] = f2v{acc[g][2], acc[g][3]};
    }
#endif
    float4 wb[KD][G];
#pragma unroll
    for (int d = 0; d < KD; ++d)
#pragma unroll
        for (int g = 0; g < G; ++g) wb[d][g] = P[(size_t)(k4b + d) * NR + j + g * KH];
    for (int k4 = k4b; k4 < k4e; k4 += KD) {
#pragma unroll
        for (int d = 0; d < KD; ++d) {
            const int kk = k4 + d;
            const float4* xr = reinterpret_cast<const float4*>(xT + 4 * KS * kk);
            const float4 x0 = xr[0], x1 = xr[1], x2 = xr[2], x3 = xr[3];   // k = 4kk .. 4kk+3, KS seqs each
            float4 w[G];
#pragma unroll
            for (int g = 0; g < G; ++g) w[g] = wb[d][g];
            const int kn = min(kk + KD, k4e - 1);   // past the range: a harmless reload of the last row
#pragma unroll
            for (int g = 0; g < G; ++g) wb[d][g] = P[(size_t)kn * NR + j + g * KH];
#pragma unroll
            for (int g = 0; g < G; ++g) {
#if TRAJ_KNET_PK
                const f2v xs[4][2] = {{f2v{x0.x, x0.y}, f2v{x0.z, x0.w}}, {f2v{x1.x, x1.y}, f2v{x1.z, x1.w}},
                                      {f2v{x2.x, x2.y}, f2v{x2.z, x2.w}}, {f2v{x3.x, x3.y}, f2v{x3.z, x3.w}}};
                const float wc[4] = {w[g].x, w[g].y, w[g].z, w[g].w};
#pragma unroll
                for (int c = 0; c < 4; ++c)
#pragma unroll
                    for (int h = 0; h < 2; ++h)
                        a2[g][h] = __builtin_elementwise_fma(xs[c][h], f2v{wc[c], wc[c]}, a2[g][h]);
#else
                acc[g][0] = fmaf(x3.x, w[g].w, fmaf(x2.x, w[g].z, fmaf(x1.x, w[g].y, fmaf(x0.x, w[g].x, acc[g][0]))));
                acc[g][1] = fmaf(x3.y, w[g].w, fmaf(x2.y, w[g].z, fmaf(x1.y, w[g].y, fmaf(x0.y, w[g].x, acc[g][1]))));
                acc[g][2] = fmaf(x3.z, w[g].w, fmaf(x2.z, w[g].z, fmaf(x1.z, w[g].y, fmaf(x0.z, w[g].x, acc[g][2]))));
                acc[g][3] = fmaf(x3.w, w[g].w, fmaf(x2.w, w[g].z, fmaf(x1.w, w[g].y, fmaf(x0.w, w[g].x, acc[g][3]))));
#endif
            }
        }
    }
#if TRAJ_KNET_PK
#pragma unroll
    for (int g = 0; g < G; ++g) {
        acc[g][0] = a2[g][0].x;
        acc[g][1] = a2[g][0].y;
        acc[g][2] = a2[g][1].x;
        acc[g][3] = a2[g][1].y;
    }
#endif
}

constexpr int K4_H = KH / 4;   // rows of 4 of every W_hh

// Timing experiments only (tools/knet_bf_stages.sh): TRAJ_BF_SKIP bit i drops stage i of
// knet_back_front_kernel (wrong results).  0 in every shipped build.
#ifndef TRAJ_BF_SKIP
#define TRAJ_BF_SKIP 0
#endif
#define BF_RUN(i) ((TRAJ_BF_SKIP & (1 << (i))) == 0)

struct NoSide {
    __device__ void operator()() const {}
};

// One output of a small dense layer (K <= 16: the whole row in quarter 0 of dense_ks) by a single
// thread, bit-identical to dense_ks: the fmaf chain in k order from the bias, then the three zero
// partials of the other quarters (which turn a -0 into +0), then ReLU.  P: packed as dense_ks reads it.
__device__ __forceinline__ float dense_one(const float* xT, int K, const float4* __restrict__ P,
                                           const float* __restrict__ bias, int N, int j, int s) {
    float acc = bias[j];
    for (int k4 = 0; 4 * k4 < K; ++k4) {
        const float4 w = P[(size_t)k4 * N + j];
        const float* x = xT + 4 * KS * k4 + s;
        acc = fmaf(x[0], w.x, acc);
        if (4 * k4 + 1 < K) acc = fmaf(x[KS], w.y, acc);
        if (4 * k4 + 2 < K) acc = fmaf(x[2 * KS], w.z, acc);
        if (4 * k4 + 3 < K) acc = fmaf(x[3 * KS], w.w, acc);
    }
    return fmaxf(__fadd_rn(acc, 0.0f), 0.0f);
}

// Dense layer: outT[j][s] = act(b[j] + sum_k xT[k][s] W[j][k]) for j < N <= KH (outT: LDS, k-major).
// xch: LDS scratch of (KQ - 1) * KH * KS floats.  Called by every thread of the workgroup.  `side` runs
// on every thread between the two barriers (after the partial sums are published, while quarter 0
// finishes): work for the threads the layer leaves idle there (units >= N).
// First half of dense_ks: quarter `part` of unit j's dot product; quarters 1..3 publish their partial
// to xch, quarter 0 keeps it (returned) for dense_finish after the barrier.
__device__ __forceinline__ float4 dense_publish(const float* xT, int K4, const float4* __restrict__ P,
                                                const float* __restrict__ bias, int N, float* xch, int t) {
    const int j = t & (KH - 1), part = t >> 7, h4 = K4 / KQ;
    float acc[1][KS] = {{0.0f, 0.0f, 0.0f, 0.0f}};
    if (j < N) {
        if (part == 0) acc[0][0] = acc[0][1] = acc[0][2] = acc[0][3] = bias[j];
        dot_ks<1>(xT, part * h4, (part + 1) * h4, P, N, j, acc);
        if (part)
            *reinterpret_cast<float4*>(xch + ((part - 1) * KH + j) * KS) =
                make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
    }
    return make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
}

__device__ __forceinline__ void dense_finish(float4 r, int N, float* outT, bool relu, const float* xch, int t) {
    const int j = t & (KH - 1), part = t >> 7;
    if (j < N && part == 0) {
#pragma unroll
        for (int q = 1; q < KQ; ++q) {
            const float4 o = *reinterpret_cast<const float4*>(xch + ((q - 1) * KH + j) * KS);
            r = make_float4(__fadd_rn(r.x, o.x), __fadd_rn(r.y, o.y), __fadd_rn(r.z, o.z), __fadd_rn(r.w, o.w));
        }
        if (relu) r = make_float4(fmaxf(r.x, 0.0f), fmaxf(r.y, 0.0f), fmaxf(r.z, 0.0f), fmaxf(r.w, 0.0f));
        *reinterpret_cast<float4*>(outT + KS * j) = r;
    }
}

template <class Side = NoSide>
__device__ __forceinline__ void dense_ks(const float* xT, int K4, const float4* __restrict__ P,
                                         const float* __restrict__ bias, int N, float* outT, bool relu, float* xch,
                                         int t, Side side = {}) {
    const int j = t & (KH - 1), part = t >> 7, h4 = K4 / KQ;
    float acc[1][KS] = {{0.0f, 0.0f, 0.0f, 0.0f}};
    if (j < N) {
        if (part == 0) acc[0][0] = acc[0][1] = acc[0][2] = acc[0][3] = bias[j];
        dot_ks<1>(xT, part * h4, (part + 1) * h4, P, N, j, acc);
        if (part)
            *reinterpret_cast<float4*>(xch + ((part - 1) * KH + j) * KS) =
                make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
    }
    __syncthreads();
    side();
    if (j < N && part == 0) {
        float4 r = make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
#pragma unroll
        for (int q = 1; q < KQ; ++q) {
            const float4 o = *reinterpret_cast<const float4*>(xch + ((q - 1) * KH + j) * KS);
            r = make_float4(__fadd_rn(r.x, o.x), __fadd_rn(r.y, o.y), __fadd_rn(r.z, o.z), __fadd_rn(r.w, o.w));
        }
        if (relu) r = make_float4(fmaxf(r.x, 0.0f), fmaxf(r.y, 0.0f), fmaxf(r.z, 0.0f), fmaxf(r.w, 0.0f));
        *reinterpret_cast<float4*>(outT + KS * j) = r;
    }
    __syncthreads();
}

// GRU cell (torch.nn.GRU, one layer, one step) for the KS sequences: xT [K][KS], hT [KH][KS] -> houtT.
// Thread (unit u, quarter q) forms its quarter's partial gates for all KS sequences, then finishes
// sequence q from the four quarters' partials (added in quarter order).  xch: LDS scratch of
// KQ * KH * 6 * KS floats.
__device__ __forceinline__ void gru_publish(const float* xT, int K4, const float* hT, const float4* __restrict__ Wi,
                                            const float* __restrict__ bi, const float4* __restrict__ Wh,
                                            const float* __restrict__ bh, float* xch, int t) {
    static_assert(KQ == KS, "one finished sequence per K quarter");
    const int u = t & (KH - 1), part = t >> 7;
    float gi[3][KS], gh[3][KS];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int q = 0; q < KS; ++q) {
            gi[g][q] = part ? 0.0f : bi[g * KH + u];
            gh[g][q] = part ? 0.0f : bh[g * KH + u];
        }
    const int hi = K4 / KQ, hh = K4_H / KQ;
    dot_ks<3>(xT, part * hi, (part + 1) * hi, Wi, 3 * KH, u, gi);
    dot_ks<3>(hT, part * hh, (part + 1) * hh, Wh, 3 * KH, u, gh);
    // publish: xch[part][u][sequence][gi r z n | gh r z n]
    float* mine = xch + (size_t)(part * KH + u) * 6 * KS;
#pragma unroll
    for (int q = 0; q < KS; ++q) {
        *reinterpret_cast<float2*>(mine + 6 * q) = make_float2(gi[0][q], gi[1][q]);
        *reinterpret_cast<float2*>(mine + 6 * q + 2) = make_float2(gi[2][q], gh[0][q]);
        *reinterpret_cast<float2*>(mine + 6 * q + 4) = make_float2(gh[1][q], gh[2][q]);
    }
}

// Second half of the GRU cell (after a barrier that follows gru_publish): thread (unit u, quarter q)
// adds the four quarters' partials of sequence q in quarter order and applies the gates.
__device__ __forceinline__ void gru_finish(const float* hT, float* houtT, const float* xch, int t) {
    const int u = t & (KH - 1), part = t >> 7;
    const int sq = part;   // the sequence this thread finishes
    float ir[3] = {0.0f, 0.0f, 0.0f}, hr[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
        const float* o = xch + (size_t)(q * KH + u) * 6 * KS + 6 * sq;
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            ir[g] = q ? __fadd_rn(ir[g], o[g]) : o[g];
            hr[g] = q ? __fadd_rn(hr[g], o[3 + g]) : o[3 + g];
        }
    }
    // ATen GRUCell: r = sigmoid(h_r + i_r), z = sigmoid(h_z + i_z), n = tanh(i_n + h_n * r), h' = (h - n) z + n
    const float r = sigmoidf_(__fadd_rn(hr[0], ir[0]));
    const float z = sigmoidf_(__fadd_rn(hr[1], ir[1]));
    const float nn = tanhf(__fadd_rn(ir[2], __fmul_rn(hr[2], r)));
    const float hv = hT[u * KS + sq];
    houtT[u * KS + sq] = __fadd_rn(__fmul_rn(__fsub_rn(hv, nn), z), nn);
}

__device__ __forceinline__ void gru_ks(const float* xT, int K4, const float* hT, const float4* __restrict__ Wi,
                                       const float* __restrict__ bi, const float4* __restrict__ Wh,
                                       const float* __restrict__ bh, float* houtT, float* xch, int t) {
    gru_publish(xT, K4, hT, Wi, bi, Wh, bh, xch, t);
    __syncthreads();
    gru_finish(hT, houtT, xch, t);
    __syncthreads();
}

__device__ __forceinline__ void front_body(KP p, traj_knet_limits L, float Ts, KNet net, int B,
                                                        const float* __restrict__ x_post, const float* __restrict__ u,
                                                        int u_sb, int u_sc, const float* __restrict__ y, int y_sb,
                                                        int y_sc, const float* __restrict__ xm,
                                                        const float* __restrict__ xs, const float* __restrict__ ym,
                                                        const float* __restrict__ ys, const float* __restrict__ um,
                                                        const float* __restrict__ us, float* hQ, const float* hSig,
                                                        float* hS, float* prior, float* dy, float* x2) {
    __shared__ __attribute__((aligned(16))) float s_h[3][KH * KS];   // h_Q, h_Sigma, h_S (inputs), k-major
    __shared__ __attribute__((aligned(16))) float s_q[KH * KS];      // new h_Q
    __shared__ __attribute__((aligned(16))) float s_g[KH * KS];      // out_Sigma
    __shared__ __attribute__((aligned(16))) float s_hs[KH * KS];     // new h_S
    __shared__ __attribute__((aligned(16))) float s_pr[64 * KS];     // prior, zero-padded to k4_
    __shared__ __attribute__((aligned(16))) float s_dy[64 * KS];     // innovation, zero-padded
    __shared__ __attribute__((aligned(16))) float s_o5[64 * KS];     // FC5 output, zero-padded
    __shared__ __attribute__((aligned(16))) float s_c1[64 * KS];     // [FC1 | FC7], zero-padded
    __shared__ __attribute__((aligned(16))) float s_x[KQ * KH * 6 * KS];   // K-quarter partial sums
    const int t = threadIdx.x, b0 = blockIdx.x * KS;
    const int nb = min(KS, B - b0);
    for (int i = t; i < 3 * KS * KH; i += KT) {   // coalesced row reads -> k-major LDS
        const int w = i / (KS * KH), r = i - w * KS * KH, s = r / KH, k = r - s * KH;
        const float* src = (w == 0) ? hQ : (w == 1 ? hSig : hS);
        s_h[w][k * KS + s] = (s < nb) ? src[(size_t)(b0 + s) * KH + k] : 0.0f;
    }
    if (t < 64 * KS) s_o5[t] = s_c1[t] = s_pr[t] = s_dy[t] = 0.0f;
    __syncthreads();
    if (t < KS) {
        float pr[6] = {0, 0, 0, 0, 0, 0}, e[5] = {0, 0, 0, 0, 0};
        if (t < nb) {
            const int b = b0 + t;
            prior_one(p, L, Ts, x_post + 6 * b, u[(size_t)b * u_sb], u[(size_t)b * u_sb + u_sc], y + (size_t)b * y_sb,
                      y_sc, xm, xs, ym, ys, um, us, pr, nullptr, e);
            for (int i = 0; i < 6; ++i) prior[6 * b + i] = pr[i];
            for (int j = 0; j < 5; ++j) dy[5 * b + j] = e[j];
        }
        for (int i = 0; i < 6; ++i) s_pr[i * KS + t] = pr[i];
        for (int j = 0; j < 5; ++j) s_dy[j * KS + t] = e[j];
    }
    __syncthreads();
    dense_ks(s_pr, k4_(net.m), net.W5, net.b5, net.dFC5, s_o5, true, s_x, t);                    // FC5 + ReLU
    gru_ks(s_o5, k4_(net.dFC5), s_h[0], net.WiQ, net.biQ, net.WhQ, net.bhQ, s_q, s_x, t);        // GRU_Q
    gru_ks(s_q, KH / 4, s_h[1], net.WiG, net.biG, net.WhG, net.bhG, s_g, s_x, t);               // GRU_Sigma
    dense_ks(s_g, KH / 4, net.W1, net.b1, net.dFC1, s_c1, true, s_x, t);                         // FC1 + ReLU
    dense_ks(s_dy, k4_(net.n), net.W7, net.b7, net.dFC7, s_c1 + KS * net.dFC1, true, s_x, t);    // FC7 + ReLU
    gru_ks(s_c1, k4_(net.dFC1 + net.dFC7), s_h[2], net.WiS, net.biS, net.WhS, net.bhS, s_hs, s_x, t);   // GRU_S
    for (int i = t; i < nb * KH; i += KT) {
        const int s = i / KH, k = i - s * KH;
        const size_t b = (size_t)(b0 + s);
        hQ[b * KH + k] = s_q[k * KS + s];
        hS[b * KH + k] = s_hs[k * KS + s];
        x2[b * 2 * KH + k] = s_g[k * KS + s];
        x2[b * 2 * KH + KH + k] = s_hs[k * KS + s];
    }
}

// FC2 = Linear(2H, dH) -> ReLU -> Linear(dH, n m) (kalman_net.py:88-95) without the [B, dH] hidden
// activation ever reaching memory.  Workgroup (slab, bblk) owns 64 sequences x HS = 64 NT hidden units
// (NT = 5: 32 slabs x 16 b-blocks = 512 workgroups at B = 1024, two per CU, every SIMD the same work):
//   1. the x2 tile [64][2H] is staged in LDS (rows padded to 260 floats);
//   2. wave w forms the TRANSPOSED hidden tile hidT[h][b] = W2a[h,:] . x2[b,:] for its 16 NT hidden units
//      and all 64 sequences on v_mfma_f32_16x16x4_f32 (exact f32): A = W2a rows streamed from L2 PD chunks
//      ahead, B = the x2 tile from LDS; NT x 4 independent 16 x 16 accumulators;
//   3. relu(hidT + b2a) stays in the accumulators and IS the B operand of the second product:
//      lane (g = l >> 4, r = l & 15) holds hidT[4g + q][r] in register q, so MFMA step q contracts over
//      h = 4g + q -- outT[j][b] = sum_h W2b[j][h] hidT[h][b] with no LDS round trip (rows j >= n m are
//      zero weights);
//   4. the four waves' outT partials are added through LDS in wave order and the workgroup writes
//      part[slab][b][0:32].
// The back kernel adds b2b and the slabs in slab order (deterministic, no atomics).  K order inside the
// MFMAs: in chunk c (16 k), lane group g takes k = 16c + 4g + e at step e, so one float4 per operand
// feeds four steps.  Blocks are spread so the b-blocks of a slab share an XCD (its W2a slab stays in
// that XCD's L2).
constexpr int F2_BT = 64, F2_LD = 2 * KH + 4, F2_RS = 68;
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float f4c(const float4& v, int e) {   // component e (constant after unrolling)
    return e == 0 ? v.x : e == 1 ? v.y : e == 2 ? v.z : v.w;
}

// hidden units per workgroup: 320 when dH allows (512 equal workgroups at B = 1024), else 256
__host__ __device__ inline int fc2_slab(int dH) { return (dH % 320 == 0) ? 320 : 256; }

template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void knet_fc2_kernel(
    int B, int dH, const float* __restrict__ x2, const float* __restrict__ W2a, const float* __restrict__ b2a,
    const float* __restrict__ W2b, int nout, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float s_t[F2_BT * F2_LD];   // x2 tile, then the wave partials
    static_assert(4 * 32 * F2_RS <= F2_BT * F2_LD, "partials fit the x2 tile");
    constexpr int HS = 64 * NT;
    const int nslab = dH / HS, nbb = (B + F2_BT - 1) / F2_BT;
    int slab, bblk;
    const int i = blockIdx.x;
    if ((nslab & 7) == 0) {
        const int xcd = i & 7, local = i >> 3;
        slab = (local / nbb) * 8 + xcd;
        bblk = local % nbb;
    } else {
        slab = i / nbb;
        bblk = i % nbb;
    }
    const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, r = l & 15;
    const int b0 = bblk * F2_BT, hw0 = slab * HS + 16 * NT * w;
    constexpr int K = 2 * KH;   // FC2 input width
#pragma unroll
    for (int it = 0; it < F2_BT * (K / 4) / 256; ++it) {   // coalesced: a row is 64 consecutive float4s
        const int q = t + 256 * it, row = q / (K / 4), c4 = q - row * (K / 4);
        const int bsrc = min(b0 + row, B - 1);           // rows past B: duplicates, never stored
        *reinterpret_cast<float4*>(s_t + row * F2_LD + 4 * c4) =
            reinterpret_cast<const float4*>(x2 + (size_t)bsrc * K)[c4];
    }
    const float* pa = W2a + (size_t)(hw0 + r) * K + 4 * g;   // h-tile ht: + 16 ht K; chunk c: + 16 c
#ifndef TRAJ_FC2_PD
#define TRAJ_FC2_PD 2
#endif
    constexpr int NC = K / 16, PD = TRAJ_FC2_PD;   // chunks; chunks of W2a loads in flight ahead of the MFMAs
    float4 wa[PD][NT];
#pragma unroll
    for (int d = 0; d < PD; ++d)
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) wa[d][ht] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 16 * d);
    __syncthreads();
    f32x4 acc[NT][4];
#pragma unroll
    for (int ht = 0; ht < NT; ++ht)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) acc[ht][bt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const float* xr = s_t + r * F2_LD + 4 * g;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const int d = c % PD;
        float4 a[NT];
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) a[ht] = wa[d][ht];
        if (c + PD < NC) {
#pragma unroll
            for (int ht = 0; ht < NT; ++ht)
                wa[d][ht] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 16 * (c + PD));
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the W2a prefetch ahead of this chunk's MFMAs
        float4 xb[4];
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) xb[bt] = *reinterpret_cast<const float4*>(xr + 16 * bt * F2_LD + 16 * c);
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int ht = 0; ht < NT; ++ht)
#pragma unroll
                for (int bt = 0; bt < 4; ++bt)
                    acc[ht][bt] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(a[ht], e), f4c(xb[bt], e), acc[ht][bt], 0, 0, 0);
    }
    // relu(hidT + b2a) in place: register q of lane (g, r) in tile (ht, bt) is hidden unit hw0 + 16 ht + 4g + q
    // of sequence b0 + 16 bt + r
#pragma unroll
    for (int ht = 0; ht < NT; ++ht) {
        const float4 bias = *reinterpret_cast<const float4*>(b2a + hw0 + 16 * ht + 4 * g);
#pragma unroll
        for (int bt = 0; bt < 4; ++bt)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[ht][bt][q] = fmaxf(__fadd_rn(acc[ht][bt][q], f4c(bias, q)), 0.0f);
    }
    // outT[j][b] over this wave's hidden units: A = W2b[j][h] (rows j = 16 jt + r), B = hidT from registers
    const float m0 = r < nout ? 1.0f : 0.0f, m1 = 16 + r < nout ? 1.0f : 0.0f;
    const float* pb0 = W2b + (size_t)min(r, nout - 1) * dH + hw0 + 4 * g;
    const float* pb1 = W2b + (size_t)min(16 + r, nout - 1) * dH + hw0 + 4 * g;
    f32x4 o[2][4];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) o[jt][bt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int ht = 0; ht < NT; ++ht) {
        float4 u0 = *reinterpret_cast<const float4*>(pb0 + 16 * ht);
        float4 u1 = *reinterpret_cast<const float4*>(pb1 + 16 * ht);
        u0.x *= m0; u0.y *= m0; u0.z *= m0; u0.w *= m0;
        u1.x *= m1; u1.y *= m1; u1.z *= m1; u1.w *= m1;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int bt = 0; bt < 4; ++bt) {
                o[0][bt] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(u0, q), acc[ht][bt][q], o[0][bt], 0, 0, 0);
                o[1][bt] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(u1, q), acc[ht][bt][q], o[1][bt], 0, 0, 0);
            }
    }
    __syncthreads();   // every wave is done with the x2 tile
    // wave partials: register q of o[jt][bt] is outT[16 jt + 4g + q][16 bt + r]
    float* red = s_t + w * 32 * F2_RS;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[(16 * jt + 4 * g + q) * F2_RS + 16 * bt + r] = o[jt][bt][q];
    __syncthreads();
    {   // thread t: sequence t >> 2, outputs 8 (t & 3) .. + 7; waves added in order
        const int bb = t >> 2, j0 = 8 * (t & 3);
        float v[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const float* p0 = s_t + (j0 + jj) * F2_RS + bb;
            v[jj] = __fadd_rn(__fadd_rn(__fadd_rn(p0[0], p0[32 * F2_RS]), p0[64 * F2_RS]), p0[96 * F2_RS]);
        }
        if (b0 + bb < B) {
            float4* dst = reinterpret_cast<float4*>(part + ((size_t)slab * B + b0 + bb) * 32 + j0);
            dst[0] = make_float4(v[0], v[1], v[2], v[3]);
            dst[1] = make_float4(v[4], v[5], v[6], v[7]);
        }
    }
}

// FC2 on the bf16 matrix cores with every f32 operand carried as three bf16 terms (the default FC2;
// traj_knet_set_fc2_mode(0) selects knet_fc2_kernel above).  x = h + m + l exactly: h = bf16(x), m = bf16(x - h),
// l = bf16(x - h - m), each residual exact in f32 (24 significand bits = 3 x 8).  A product a b is formed from the
// six bf16 products h_a h_b, h_a m_b, m_a h_b, h_a l_b, l_a h_b, m_a m_b -- each exact in the f32 accumulator --
// and the three dropped ones (m_a l_b, l_a m_b, l_a l_b) are below 2^-23 |a b|, the size of one f32 rounding
// of the product.  So the sums carry f32 accuracy (f32 accumulation, different summation order), at six
// v_mfma_f32_16x16x32_bf16 (16 cycles, 16,384 FLOP each) per 16 x 16 x 32 block where the f32 form needs eight
// v_mfma_f32_16x16x4_f32 (32 cycles, 2,048 FLOP each): 96 against 256 matrix-core cycles.
// Same tiling as knet_fc2_kernel (64 sequences x 64 NT hidden units per workgroup, the x2 tile in LDS, wave w's
// transposed hidden tile in registers as the second product's B operand), K steps of 32:
//   A = W2a rows: lane (r, g) of h-tile ht, K step c holds W2a[h0 + 16 ht + r][32 c + 8 g .. + 7] (two float4
//       loads, one K step ahead), split in registers;
//   B = x2 from the LDS tile: lane (r, g) holds x2[b0 + 16 bt + r][32 c + 8 g .. + 7], split in registers;
//   second product, K step s over the tile pair (2s, 2s + 1): B element e of lane (r, g) = hidT[16 (2s + e / 4)
//       + 4 g + e % 4][16 bt + r] = register e % 4 of accumulator (2s + e / 4, bt), so A element e = W2b[j][that
//       same h] (two float4 runs of W2b's row); an odd NT's last step has a zero upper half.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// (the subtractions may pair into v_pk_add_f32: measured 35.0 us for the FC2 launch against 37.4 us with single
// v_sub_f32 forced by inline asm)
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r1 = __fsub_rn(x, (float)h);
    m = (__bf16)r1;
    l = (__bf16)__fsub_rn(r1, (float)m);
}

__device__ __forceinline__ void split3(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        __bf16 vh, vm, vl;
        split3(v[e], vh, vm, vl);
        h[e] = vh;
        m[e] = vm;
        l[e] = vl;
    }
}

__device__ __forceinline__ void split3(const float4& a, const float4& b, bf16x8& h, bf16x8& m, bf16x8& l) {
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    split3(v, h, m, l);
}

// acc += a b over one K step of 32, the six kept products, smallest first
__device__ __forceinline__ f32x4 mfma6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                       const bf16x8& bm, const bf16x8& bl, f32x4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
}

// The three-term kernels' second half: relu(hidT + b2a) in the accumulators, the second product on the bf16 matrix
// cores (B = the accumulators, A = W2b split in registers), the four waves' partials added in wave order through LDS
// (s_red: 4 x 32 x (16 BT + 4) floats, free once every wave is past its reads of the tile), part[slab][b][0:32]
// written.  BT: 16-sequence tiles per workgroup.
template <int NT, int BT = 4>
__device__ __forceinline__ void fc2x_epilogue(f32x4 (&acc)[NT][BT], const float* __restrict__ b2a,
                                              const float* __restrict__ W2b, int dH, int nout, int hw0, int B, int b0,
                                              int slab, float* s_red, float* __restrict__ part) {
    constexpr int RS = 16 * BT + 4;   // (F2_RS at BT = 4)
    const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, r = l & 15;
    // relu(hidT + b2a) in place (register q of lane (g, r) in tile (ht, bt): unit hw0 + 16 ht + 4 g + q, sequence
    // b0 + 16 bt + r)
#pragma unroll
    for (int ht = 0; ht < NT; ++ht) {
        const float4 bias = *reinterpret_cast<const float4*>(b2a + hw0 + 16 * ht + 4 * g);
#pragma unroll
        for (int bt = 0; bt < BT; ++bt)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[ht][bt][q] = fmaxf(__fadd_rn(acc[ht][bt][q], f4c(bias, q)), 0.0f);
    }
    // outT[j][b] = sum over this wave's units of W2b[j][h] hidT[h][b] (rows j = 16 jt + r; rows >= nout: zero)
    const float m0 = r < nout ? 1.0f : 0.0f, m1 = 16 + r < nout ? 1.0f : 0.0f;
    const float* pb[2] = {W2b + (size_t)min(r, nout - 1) * dH + hw0 + 4 * g,
                          W2b + (size_t)min(16 + r, nout - 1) * dH + hw0 + 4 * g};
    const float mk[2] = {m0, m1};
    f32x4 o[2][BT];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int bt = 0; bt < BT; ++bt) o[jt][bt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int s = 0; s < (NT + 1) / 2; ++s) {
        constexpr float z = 0.0f;
        const bool hi2 = 2 * s + 1 < NT;   // the step's upper tile exists
        bf16x8 wh[2], wm[2], wl[2];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            float4 u0 = *reinterpret_cast<const float4*>(pb[jt] + 32 * s);
            float4 u1 = hi2 ? *reinterpret_cast<const float4*>(pb[jt] + 32 * s + 16) : make_float4(z, z, z, z);
            const float v[8] = {u0.x * mk[jt], u0.y * mk[jt], u0.z * mk[jt], u0.w * mk[jt],
                                u1.x * mk[jt], u1.y * mk[jt], u1.z * mk[jt], u1.w * mk[jt]};
            split3(v, wh[jt], wm[jt], wl[jt]);
        }
#pragma unroll
        for (int bt = 0; bt < BT; ++bt) {
            float v[8];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = acc[2 * s][bt][e];
                v[4 + e] = hi2 ? acc[hi2 ? 2 * s + 1 : 2 * s][bt][e] : 0.0f;
            }
            bf16x8 bh, bm, bl;
            split3(v, bh, bm, bl);
#pragma unroll
            for (int jt = 0; jt < 2; ++jt) o[jt][bt] = mfma6(wh[jt], wm[jt], wl[jt], bh, bm, bl, o[jt][bt]);
        }
    }
    __syncthreads();   // every wave is done with the tile in LDS
    float* red = s_red + w * 32 * RS;
#pragma unroll
    for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int bt = 0; bt < BT; ++bt)
#pragma unroll
            for (int q = 0; q < 4; ++q) red[(16 * jt + 4 * g + q) * RS + 16 * bt + r] = o[jt][bt][q];
    __syncthreads();
    {   // thread t: sequence t / TPS, outputs JW (t % TPS) .. + JW - 1; waves added in order
        constexpr int SEQ = 16 * BT, TPS = 256 / SEQ, JW = 32 / TPS;
        const int bb = t / TPS, j0 = JW * (t % TPS);
        float v[JW];
#pragma unroll
        for (int jj = 0; jj < JW; ++jj) {
            const float* p0 = s_red + (j0 + jj) * RS + bb;
            v[jj] = __fadd_rn(__fadd_rn(__fadd_rn(p0[0], p0[32 * RS]), p0[64 * RS]), p0[96 * RS]);
        }
        if (b0 + bb < B) {
            float4* dst = reinterpret_cast<float4*>(part + ((size_t)slab * B + b0 + bb) * 32 + j0);
#pragma unroll
            for (int k = 0; k < JW / 4; ++k) dst[k] = make_float4(v[4 * k], v[4 * k + 1], v[4 * k + 2], v[4 * k + 3]);
        }
    }
}

template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void knet_fc2x_kernel(
    int B, int dH, const float* __restrict__ x2, const float* __restrict__ W2a, const float* __restrict__ b2a,
    const float* __restrict__ W2b, int nout, float* __restrict__ part) {
    __shared__ __attribute__((aligned(16))) float s_t[F2_BT * F2_LD];   // x2 tile, then the wave partials
    constexpr int HS = 64 * NT;
    const int nslab = dH / HS, nbb = (B + F2_BT - 1) / F2_BT;
    int slab, bblk;
    const int i = blockIdx.x;
    if ((nslab & 7) == 0) {   // the b-blocks of a slab on one XCD (its W2a slab stays in that L2)
        const int xcd = i & 7, local = i >> 3;
        slab = (local / nbb) * 8 + xcd;
        bblk = local % nbb;
    } else {
        slab = i / nbb;
        bblk = i % nbb;
    }
    const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, r = l & 15;
    const int b0 = bblk * F2_BT, hw0 = slab * HS + 16 * NT * w;
    constexpr int K = 2 * KH;
#pragma unroll
    for (int it = 0; it < F2_BT * (K / 4) / 256; ++it) {
        const int q = t + 256 * it, row = q / (K / 4), c4 = q - row * (K / 4);
        const int bsrc = min(b0 + row, B - 1);   // rows past B: duplicates, never stored
        *reinterpret_cast<float4*>(s_t + row * F2_LD + 4 * c4) = reinterpret_cast<const float4*>(x2 + (size_t)bsrc * K)[c4];
    }
    const float* pa = W2a + (size_t)(hw0 + r) * K + 8 * g;   // h-tile ht: + 16 ht K; K step c: + 32 c
    constexpr int NC = K / 32;
    float4 an[NT][2];
    auto load_a = [&](int c) {
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) {
            an[ht][0] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 32 * c);
            an[ht][1] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 32 * c + 4);
        }
    };
    load_a(0);
    __syncthreads();
    f32x4 acc[NT][4];
#pragma unroll
    for (int ht = 0; ht < NT; ++ht)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) acc[ht][bt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const float* xr = s_t + r * F2_LD + 8 * g;
    for (int c = 0; c < NC; ++c) {
        bf16x8 ah[NT], am[NT], al[NT];
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) split3(an[ht][0], an[ht][1], ah[ht], am[ht], al[ht]);
        if (c + 1 < NC) load_a(c + 1);
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
            const float4* xp = reinterpret_cast<const float4*>(xr + 16 * bt * F2_LD + 32 * c);
            bf16x8 bh, bm, bl;
            split3(xp[0], xp[1], bh, bm, bl);
#pragma unroll
            for (int ht = 0; ht < NT; ++ht) acc[ht][bt] = mfma6(ah[ht], am[ht], al[ht], bh, bm, bl, acc[ht][bt]);
        }
    }
    fc2x_epilogue<NT>(acc, b2a, W2b, dH, nout, hw0, B, b0, slab, s_t, part);
}

// The three-term FC2 with the x2 tile split ONCE per workgroup (knet_fc2x_kernel has every wave split all 64 sequences'
// values at every K step): the tile's three bf16 planes in LDS, one K half at a time (52 KB, so two workgroups still
// share a CU), W2a split in registers as in knet_fc2x_kernel.  Same terms, same summation order, bit for bit.
constexpr int F2_HK = KH;            // K columns per half
constexpr int F2_BLD = F2_HK + 8;    // bf16 per LDS plane row (272 B: rows 4 banks apart)

template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void knet_fc2y_kernel(
    int B, int dH, const float* __restrict__ x2, const float* __restrict__ W2a, const float* __restrict__ b2a,
    const float* __restrict__ W2b, int nout, float* __restrict__ part) {
    constexpr int PL = F2_BT * F2_BLD;
    __shared__ __attribute__((aligned(16))) __bf16 s_b[3 * PL];   // one K half of the tile: hi, mid, lo planes
    static_assert(4 * 32 * F2_RS * sizeof(float) <= sizeof(s_b), "partials fit the planes");
    constexpr int HS = 64 * NT;
    const int nslab = dH / HS, nbb = (B + F2_BT - 1) / F2_BT;
    int slab, bblk;
    const int i = blockIdx.x;
    if ((nslab & 7) == 0) {
        const int xcd = i & 7, local = i >> 3;
        slab = (local / nbb) * 8 + xcd;
        bblk = local % nbb;
    } else {
        slab = i / nbb;
        bblk = i % nbb;
    }
    const int t = threadIdx.x, w = t >> 6, l = t & 63, g = l >> 4, r = l & 15;
    const int b0 = bblk * F2_BT, hw0 = slab * HS + 16 * NT * w;
    constexpr int K = 2 * KH, NC = K / 32;
    const float* pa = W2a + (size_t)(hw0 + r) * K + 8 * g;
    float4 an[NT][2];
    auto load_a = [&](int c) {
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) {
            an[ht][0] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 32 * c);
            an[ht][1] = *reinterpret_cast<const float4*>(pa + (size_t)16 * ht * K + 32 * c + 4);
        }
    };
    // half hf of the tile, split: thread t takes float4 q = t + 256 it (row q / 32, columns hf 128 + 4 (q % 32) .. + 3)
    auto stage = [&](int hf) {
#pragma unroll 4
        for (int it = 0; it < F2_BT * (F2_HK / 4) / 256; ++it) {
            const int q = t + 256 * it, row = q / (F2_HK / 4), c4 = q - row * (F2_HK / 4);
            const int bsrc = min(b0 + row, B - 1);   // rows past B: duplicates, never stored
            const float4 v = reinterpret_cast<const float4*>(x2 + (size_t)bsrc * K + hf * F2_HK)[c4];
            const float vv[4] = {v.x, v.y, v.z, v.w};
            typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
            bf16x4 h, m, lo;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                __bf16 a0, a1, a2;
                split3(vv[e], a0, a1, a2);
                h[e] = a0;
                m[e] = a1;
                lo[e] = a2;
            }
            const int o = row * F2_BLD + 4 * c4;
            *reinterpret_cast<bf16x4*>(s_b + o) = h;
            *reinterpret_cast<bf16x4*>(s_b + PL + o) = m;
            *reinterpret_cast<bf16x4*>(s_b + 2 * PL + o) = lo;
        }
    };
    load_a(0);
    stage(0);
    __syncthreads();
    f32x4 acc[NT][4];
#pragma unroll
    for (int ht = 0; ht < NT; ++ht)
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) acc[ht][bt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    const __bf16* xr = s_b + r * F2_BLD + 8 * g;
    for (int c = 0; c < NC; ++c) {
        if (c == NC / 2) {   // second K half
            __syncthreads();
            stage(1);
            __syncthreads();
        }
        bf16x8 ah[NT], am[NT], al[NT];
#pragma unroll
        for (int ht = 0; ht < NT; ++ht) split3(an[ht][0], an[ht][1], ah[ht], am[ht], al[ht]);
        if (c + 1 < NC) load_a(c + 1);
        const int cc = c & (NC / 2 - 1);
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
            const __bf16* bp = xr + 16 * bt * F2_BLD + 32 * cc;
            const bf16x8 bh = *reinterpret_cast<const bf16x8*>(bp);
            const bf16x8 bm = *reinterpret_cast<const bf16x8*>(bp + PL);
            const bf16x8 bl = *reinterpret_cast<const bf16x8*>(bp + 2 * PL);
#pragma unroll
            for (int ht = 0; ht < NT; ++ht) acc[ht][bt] = mfma6(ah[ht], am[ht], al[ht], bh, bm, bl, acc[ht][bt]);
        }
    }
    fc2x_epilogue<NT>(acc, b2a, W2b, dH, nout, hw0, B, b0, slab, reinterpret_cast<float*>(s_b), part);
}

__device__ __forceinline__ void back_body(KNet net, int B, const float* __restrict__ x2,
                                                       const float* __restrict__ part, int nslab,
                                                       const float* __restrict__ prior, const float* __restrict__ dy,
                                                       float* hSig, float* x_post, float* out, int o_sb, int o_sc,
                                                       float* KG_out) {
    __shared__ __attribute__((aligned(16))) float s_a[(KH + 64) * KS];    // [h_S | KG | 0]: FC3's input
    __shared__ __attribute__((aligned(16))) float s_b[(KH + 64) * KS];    // [out_Sigma | FC3 | 0]: FC4's input
    __shared__ __attribute__((aligned(16))) float s_o[KH * KS];           // FC4 output (new h_Sigma)
    __shared__ __attribute__((aligned(16))) float s_x[(KQ - 1) * KH * KS];   // K-quarter partial sums
    __shared__ float s_red[KS][32][4];
    const int t = threadIdx.x, b0 = blockIdx.x * KS;
    const int nb = min(KS, B - b0);
    const int nm = net.n * net.m;
    for (int i = t; i < KS * 2 * KH; i += KT) {
        const int s = i / (2 * KH), k = i - s * 2 * KH;
        const float v = (s < nb) ? x2[(size_t)(b0 + s) * 2 * KH + k] : 0.0f;
        if (k < KH) s_b[k * KS + s] = v;
        else s_a[(k - KH) * KS + s] = v;
    }
    for (int i = t; i < 64 * KS; i += KT) s_b[KH * KS + i] = 0.0f;
    for (int i = t; i < 32 * KS; i += KT) s_a[(KH + 32) * KS + i] = 0.0f;
    {   // KG = b2b + sum over FC2's slabs: thread (s, j, q) sums the slabs sl = q mod 4
        const int s = t >> 7, j = (t >> 2) & 31, q = t & 3;
        float a = 0.0f;
        if (s < nb) {
            const float* pp = part + ((size_t)b0 + s) * 32 + j;
#pragma unroll 8
            for (int sl = q; sl < nslab; sl += 4) a = __fadd_rn(a, pp[(size_t)sl * B * 32]);
        }
        s_red[s][j][q] = a;
    }
    __syncthreads();
    if (t < KS * 32) {
        const int s = t >> 5, j = t & 31;
        float v = 0.0f;
        if (j < nm && s < nb) {
            v = __fadd_rn(net.b2b[j], __fadd_rn(__fadd_rn(s_red[s][j][0], s_red[s][j][1]),
                                                __fadd_rn(s_red[s][j][2], s_red[s][j][3])));
            if (KG_out) KG_out[(size_t)(b0 + s) * nm + j] = v;
        }
        s_a[(KH + j) * KS + s] = v;
    }
    __syncthreads();
    // FC3 + ReLU on cat(h_S, out_FC2); FC4 + ReLU on cat(out_Sigma, out_FC3) = the new h_Sigma
    dense_ks(s_a, k4_(KH + nm), net.W3, net.b3, net.dFC3, s_b + KH * KS, true, s_x, t);
    dense_ks(s_b, k4_(KH + net.dFC3), net.W4, net.b4, KH, s_o, true, s_x, t);
    for (int i = t; i < nb * KH; i += KT) {
        const int s = i / KH, k = i - s * KH;
        hSig[(size_t)(b0 + s) * KH + k] = s_o[k * KS + s];
    }
    if (t < nb) {   // posterior (kalman_net.py:169-178), as knet_update_kernel
        const int b = b0 + t;
        const float gamma = sigmoidf_(net.logit[0]);
        for (int i = 0; i < net.m; ++i) {
            float sacc = 0.0f;
            for (int j = 0; j < net.n; ++j)
                sacc = __fadd_rn(sacc, __fmul_rn(s_a[(KH + net.n * i + j) * KS + t], dy[5 * b + j]));
            const float v = __fadd_rn(prior[6 * b + i], __fmul_rn(gamma, sacc));
            x_post[6 * b + i] = v;
            if (out) out[(size_t)b * o_sb + (size_t)i * o_sc] = v;
        }
    }
}

__global__ __launch_bounds__(KT) void knet_front_kernel(KP p, traj_knet_limits L, float Ts, KNet net, int B,
                                                        const float* x_post, const float* u, int u_sb, int u_sc,
                                                        const float* y, int y_sb, int y_sc, const float* xm,
                                                        const float* xs, const float* ym, const float* ys,
                                                        const float* um, const float* us, float* hQ, const float* hSig,
                                                        float* hS, float* prior, float* dy, float* x2) {
    front_body(p, L, Ts, net, B, x_post, u, u_sb, u_sc, y, y_sb, y_sc, xm, xs, ym, ys, um, us, hQ, hSig, hS, prior, dy,
               x2);
}

__global__ __launch_bounds__(KT) void knet_back_kernel(KNet net, int B, const float* x2, const float* part, int nslab,
                                                       const float* prior, const float* dy, float* hSig, float* x_post,
                                                       float* out, int o_sb, int o_sc, float* KG_out) {
    back_body(net, B, x2, part, nslab, prior, dy, hSig, x_post, out, o_sb, o_sc, KG_out);
}

// back(t) and front(t + 1) in one launch: a workgroup finishes step t of its four sequences and goes
// straight on to step t + 1 -- one launch and one workgroup start per step fewer, h_Sigma(t) handed
// over in LDS, and the posterior x_post(t) (it needs FC2's output, not FC3/FC4) plus step t + 1's prior
// computed by four threads that FC3 leaves idle (units >= d_fc3) while the others run FC3.  Each
// workgroup reads and writes only its own sequences' rows.  Bit-identical to back(t) + front(t + 1).
__global__ __launch_bounds__(KT) void knet_back_front_kernel(KNet net, int B, const float* __restrict__ part,
                                                             int nslab, float* __restrict__ out, int o_sb, int o_sc,
                                                             KP p, traj_knet_limits L, float Ts,
                                                             const float* __restrict__ u, int u_sb, int u_sc,
                                                             const float* __restrict__ y, int y_sb, int y_sc,
                                                             const float* __restrict__ xm, const float* __restrict__ xs,
                                                             const float* __restrict__ ym, const float* __restrict__ ys,
                                                             const float* __restrict__ um, const float* __restrict__ us,
                                                             float* __restrict__ hQ, float* __restrict__ hSig,
                                                             float* __restrict__ hS, float* __restrict__ x_post,
                                                             float* __restrict__ prior, float* __restrict__ dy,
                                                             float* __restrict__ x2) {
    __shared__ __attribute__((aligned(16))) float s_a[(KH + 64) * KS];    // [h_S(t) | KG | 0]: FC3's input
    __shared__ __attribute__((aligned(16))) float s_b[(KH + 64) * KS];    // [out_Sigma(t) | FC3 | 0]: FC4's input
    __shared__ __attribute__((aligned(16))) float s_o[KH * KS];           // FC4 output = h_Sigma(t)
    __shared__ __attribute__((aligned(16))) float s_hq[KH * KS];          // h_Q(t)
    __shared__ __attribute__((aligned(16))) float s_q[KH * KS];           // h_Q(t + 1)
    __shared__ __attribute__((aligned(16))) float s_g[KH * KS];           // out_Sigma(t + 1)
    __shared__ __attribute__((aligned(16))) float s_hs[KH * KS];          // h_S(t + 1)
    __shared__ __attribute__((aligned(16))) float s_pr[64 * KS];          // prior(t + 1), zero-padded
    __shared__ __attribute__((aligned(16))) float s_dy[64 * KS];          // innovation(t + 1), zero-padded
    __shared__ __attribute__((aligned(16))) float s_o5[64 * KS];          // FC5 output, zero-padded
    __shared__ __attribute__((aligned(16))) float s_c1[64 * KS];          // [FC1 | FC7], zero-padded
    __shared__ __attribute__((aligned(16))) float s_x[KQ * KH * 6 * KS];  // K-quarter partial sums
    __shared__ float s_red[KS][32][4];
    __shared__ __attribute__((aligned(16))) float s_x4[(KQ - 1) * KH * KS];  // FC4's partials (beside GRU_Q's)
    const int t = threadIdx.x, b0 = blockIdx.x * KS;
    const int nb = min(KS, B - b0);
    const int nm = net.n * net.m;
    // ---- staging: x2(t) = [out_Sigma | h_S] and h_Q(t), k-major
    for (int i = t; i < KS * 2 * KH; i += KT) {
        const int s = i / (2 * KH), k = i - s * 2 * KH;
        const float v = (s < nb) ? x2[(size_t)(b0 + s) * 2 * KH + k] : 0.0f;
        if (k < KH) s_b[k * KS + s] = v;
        else s_a[(k - KH) * KS + s] = v;
    }
    for (int i = t; i < KS * KH; i += KT) {
        const int s = i / KH, k = i - s * KH;
        s_hq[k * KS + s] = (s < nb) ? hQ[(size_t)(b0 + s) * KH + k] : 0.0f;
    }
    for (int i = t; i < 64 * KS; i += KT) s_b[KH * KS + i] = 0.0f;
    for (int i = t; i < 32 * KS; i += KT) s_a[(KH + 32) * KS + i] = 0.0f;
    if (t < 64 * KS) s_o5[t] = s_c1[t] = s_pr[t] = s_dy[t] = 0.0f;
    {   // KG = b2b + sum over FC2's slabs: thread (s, j, q) sums the slabs sl = q mod 4
        const int s = t >> 7, j = (t >> 2) & 31, q = t & 3;
        float a = 0.0f;
        if (s < nb) {
            const float* pp = part + ((size_t)b0 + s) * 32 + j;
            if (BF_RUN(0))
#pragma unroll 8
                for (int sl = q; sl < nslab; sl += 4) a = __fadd_rn(a, pp[(size_t)sl * B * 32]);
        }
        s_red[s][j][q] = a;
    }
    __syncthreads();
    if (t < KS * 32) {
        const int s = t >> 5, j = t & 31;
        float v = 0.0f;
        if (j < nm && s < nb)
            v = __fadd_rn(net.b2b[j], __fadd_rn(__fadd_rn(s_red[s][j][0], s_red[s][j][1]),
                                                __fadd_rn(s_red[s][j][2], s_red[s][j][3])));
        s_a[(KH + j) * KS + s] = v;
    }
    __syncthreads();
    // ---- posterior x_post(t) (kalman_net.py:169-178) and step t + 1's prior (:145-162): threads
    // KT - KS .. KT - 1 (K quarter 3, units 124..127: idle in FC3), overlapping FC3
    if (t >= KT - KS) {
        const int s = t - (KT - KS);
        float pr[6] = {0, 0, 0, 0, 0, 0}, e[5] = {0, 0, 0, 0, 0};
        if (s < nb && BF_RUN(1)) {
            const int b = b0 + s;
            const float gamma = sigmoidf_(net.logit[0]);
            float xp[6];
            for (int i = 0; i < 6; ++i) {
                float sacc = 0.0f;
                for (int j = 0; j < 5; ++j)
                    sacc = __fadd_rn(sacc, __fmul_rn(s_a[(KH + 5 * i + j) * KS + s], dy[5 * b + j]));
                xp[i] = __fadd_rn(prior[6 * b + i], __fmul_rn(gamma, sacc));
                x_post[6 * b + i] = xp[i];
                out[(size_t)b * o_sb + (size_t)i * o_sc] = xp[i];
            }
            prior_one(p, L, Ts, xp, u[(size_t)b * u_sb], u[(size_t)b * u_sb + u_sc], y + (size_t)b * y_sb, y_sc, xm,
                      xs, ym, ys, um, us, pr, nullptr, e);
            for (int i = 0; i < 6; ++i) prior[6 * b + i] = pr[i];
            for (int j = 0; j < 5; ++j) dy[5 * b + j] = e[j];
        }
        for (int i = 0; i < 6; ++i) s_pr[i * KS + s] = pr[i];
        for (int j = 0; j < 5; ++j) s_dy[j * KS + s] = e[j];
    }
    // ---- back(t): FC3 + ReLU on cat(h_S, out_FC2); FC4 + ReLU on cat(out_Sigma, out_FC3) = h_Sigma(t).
    // FC3 has at most 64 units, so units 64..127 are idle once its partials are published: there they
    // run step t + 1's FC5 (on the prior) and FC7 (on the innovation), one output per thread, instead of
    // two more layer stages after FC4.
    // (fc57's loop strides over any number of FC5 / FC7 outputs: in_mult 10's 60 + 5 units included)
    const bool side = net.dFC3 <= 64 && net.m <= 16 && net.n <= 16;
    auto fc57 = [&]() {
        if (!side || (t & (KH - 1)) < 64) return;
        const int i = (t >> 7) * 64 + (t & 63);
        for (int o = i; o < (net.dFC5 + net.dFC7) * KS; o += KT / 2) {
            const int s = o & (KS - 1), unit = o / KS;
            if (unit < net.dFC5) s_o5[unit * KS + s] = dense_one(s_pr, net.m, net.W5, net.b5, net.dFC5, unit, s);
            else {
                const int v = unit - net.dFC5;
                s_c1[(net.dFC1 + v) * KS + s] = dense_one(s_dy, net.n, net.W7, net.b7, net.dFC7, v, s);
            }
        }
    };
    if (BF_RUN(2)) dense_ks(s_a, k4_(KH + nm), net.W3, net.b3, net.dFC3, s_b + KH * KS, true, s_x, t, fc57);
    // ---- front(t + 1): FC5, GRU_Q, GRU_Sigma (on h_Sigma(t) in LDS), FC1, FC7, GRU_S (on h_S(t) = s_a[0, KH)).
    // With FC5 done above, GRU_Q(t + 1) does not wait for FC4(t): the two share one stage (both
    // publish their quarter partials, one barrier, both finish).
    if (side && BF_RUN(3)) {
        const float4 r4 = dense_publish(s_b, k4_(KH + net.dFC3), net.W4, net.b4, KH, s_x4, t);
        gru_publish(s_o5, k4_(net.dFC5), s_hq, net.WiQ, net.biQ, net.WhQ, net.bhQ, s_x, t);
        __syncthreads();
        dense_finish(r4, KH, s_o, true, s_x4, t);
        gru_finish(s_hq, s_q, s_x, t);
        __syncthreads();
    } else if (!side) {
        dense_ks(s_b, k4_(KH + net.dFC3), net.W4, net.b4, KH, s_o, true, s_x, t);
        dense_ks(s_pr, k4_(net.m), net.W5, net.b5, net.dFC5, s_o5, true, s_x, t);                // FC5 + ReLU
        gru_ks(s_o5, k4_(net.dFC5), s_hq, net.WiQ, net.biQ, net.WhQ, net.bhQ, s_q, s_x, t);      // GRU_Q
    }
    for (int i = t; i < nb * KH; i += KT) {
        const int s = i / KH, k = i - s * KH;
        hSig[(size_t)(b0 + s) * KH + k] = s_o[k * KS + s];
    }
    if (BF_RUN(4)) gru_ks(s_q, KH / 4, s_o, net.WiG, net.biG, net.WhG, net.bhG, s_g, s_x, t);     // GRU_Sigma
    if (BF_RUN(5)) dense_ks(s_g, KH / 4, net.W1, net.b1, net.dFC1, s_c1, true, s_x, t);           // FC1 + ReLU
    if (!side) dense_ks(s_dy, k4_(net.n), net.W7, net.b7, net.dFC7, s_c1 + KS * net.dFC1, true, s_x, t);   // FC7
    if (BF_RUN(6)) gru_ks(s_c1, k4_(net.dFC1 + net.dFC7), s_a, net.WiS, net.biS, net.WhS, net.bhS, s_hs, s_x, t);  // GRU_S
    for (int i = t; i < nb * KH; i += KT) {
        const int s = i / KH, k = i - s * KH;
        const size_t b = (size_t)(b0 + s);
        hQ[b * KH + k] = s_q[k * KS + s];
        hS[b * KH + k] = s_hs[k * KS + s];
        x2[b * 2 * KH + k] = s_g[k * KS + s];
        x2[b * 2 * KH + KH + k] = s_hs[k * KS + s];
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

// traj_knet_set_fc2_mode: 2 = knet_fc2y_kernel (three-term bf16 operands, the tile split once per workgroup; the
// default), 1 = knet_fc2x_kernel (the same terms and sums, every wave splitting the tile), 0 = knet_fc2_kernel (f32).
static std::atomic<int> g_fc2_mode{2};

// FC2 launch in the mode of traj_knet_set_fc2_mode
static int fc2_launch(const traj_knet_net* net, int B, const float* x2, float* ws, void* stream) {
    const int hs = fc2_slab(net->d_fc2h), nslab = net->d_fc2h / hs, nbb = nblk(B, F2_BT);
    const int mode = g_fc2_mode.load(std::memory_order_relaxed);
    auto kern = mode == 2 ? (hs == 320 ? knet_fc2y_kernel<5> : knet_fc2y_kernel<4>)
              : mode == 1 ? (hs == 320 ? knet_fc2x_kernel<5> : knet_fc2x_kernel<4>)
                          : (hs == 320 ? knet_fc2_kernel<5> : knet_fc2_kernel<4>);
    hipLaunchKernelGGL(kern, dim3(nslab * nbb), dim3(256), 0, (hipStream_t)stream, B, net->d_fc2h, x2, net->fc2a_w,
                       net->fc2a_b, net->fc2b_w, net->n * net->m, ws);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

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

int traj_knet_rollout_windows(int T, int H, int t0, int step) {
    if (T < 0 || H < 1 || t0 < 0 || step < 1) return -1;
    const int end = T - H;   // range(t0, T - H, step)
    return end > t0 ? (end - t0 + step - 1) / step : 0;
}

int traj_knet_rollout_eval_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, int B, int T,
                               int H, int t0, int step, int nwin, const float* x_est, int e_sb, int e_sc, int e_st,
                               const float* x_mean, const float* x_std, const float* u, const float* x_gt, float* ade,
                               float* fde, float* err_profile, float* pred, void* stream) {
    if (!p || !lim || B < 0 || T < 0 || H < 1 || t0 < 0 || step < 1 || nwin < 0) return TRAJ_E_ARG;
    // every window's inputs u[:, :, t .. t + H - 1] (and, when scored, its ground truth x_gt[:, :, t + 1 .. t + H])
    // lie inside the sequence
    if (nwin > 0 && (long long)t0 + (long long)(nwin - 1) * step + H > (long long)T - (x_gt ? 1 : 0))
        return TRAJ_E_ARG;
    if ((long long)B * nwin > 0x7fffffffLL || e_sb < 0 || e_sc < 0 || e_st < 0) return TRAJ_E_ARG;
    if (B == 0 || nwin == 0) return TRAJ_OK;
    if (!x_est || !u || (!x_mean) != (!x_std)) return TRAJ_E_ARG;
    if (x_gt ? (!ade || !fde) : !pred) return TRAJ_E_ARG;
    KP k{(float)p->Cm1, (float)p->Cm2, (float)p->Cr0, (float)p->Cr2, (float)p->Br, (float)p->Cr, (float)p->Dr,
         (float)p->Bf,  (float)p->Cf,  (float)p->Df,  (float)p->m,   (float)p->Iz, (float)p->lf, (float)p->lr,
         (float)p->maxAlpha, (float)p->vx_zero};
    hipLaunchKernelGGL(knet_rollout_kernel, dim3(nblk((long long)B * nwin, 64)), dim3(64), 0, (hipStream_t)stream, k,
                       *lim, Ts, B, T, H, t0, step, nwin, x_est, e_sb, e_sc, e_st, x_mean, x_std, u, x_gt, ade, fde,
                       x_gt ? err_profile : nullptr, pred);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

static bool knet_ok(const traj_knet_net* w) {
    // FC5 / [FC1 | FC7] outputs live in 64-wide zero-padded LDS rows: in_mult 5 and 10 (d_fc5 30 / 60)
    return w && w->m == 6 && w->n == 5 && w->hidden == KH && w->d_fc5 > 0 && w->d_fc5 <= 64 && w->d_fc1 > 0 &&
           w->d_fc7 > 0 && w->d_fc1 + w->d_fc7 <= 64 && w->d_fc3 > 0 && w->d_fc3 <= 64 && w->fc5_w && w->fc5_b &&
           w->gru_q_wih && w->gru_q_bih && w->gru_q_whh && w->gru_q_bhh && w->gru_sigma_wih && w->gru_sigma_bih &&
           w->gru_sigma_whh && w->gru_sigma_bhh && w->fc1_w && w->fc1_b && w->fc7_w && w->fc7_b && w->gru_s_wih &&
           w->gru_s_bih && w->gru_s_whh && w->gru_s_bhh && w->fc3_w && w->fc3_b && w->fc4_w && w->fc4_b && w->innov_logit &&
           w->d_fc2h > 0 && w->d_fc2h % 256 == 0 && w->fc2a_w && w->fc2a_b && w->fc2b_w && w->fc2b_b;
}
static KNet knet_args(const traj_knet_net* w, const float* packed) {
    const PackPlan pl = pack_plan(w);
    auto P = [&](int i) { return reinterpret_cast<const float4*>(packed + pl.off[i]); };
    return KNet{w->m,     w->n,     w->d_fc5, w->d_fc1, w->d_fc7, w->d_fc3, w->fc5_b,  w->gru_q_bih, w->gru_q_bhh,
                w->gru_sigma_bih, w->gru_sigma_bhh, w->fc1_b, w->fc7_b, w->gru_s_bih, w->gru_s_bhh, w->fc3_b,
                w->fc4_b, w->innov_logit, w->fc2b_b, P(0), P(1), P(2), P(3), P(4), P(5), P(6), P(7), P(8), P(9), P(10)};
}

size_t traj_knet_packed_bytes(const traj_knet_net* net) {
    if (!knet_ok(net)) return 0;
    return pack_plan(net).off[11] * sizeof(float);
}

int traj_knet_pack_f32(const traj_knet_net* net, float* packed, size_t bytes, void* stream) {
    if (!net || !packed) return TRAJ_E_ARG;
    if (!knet_ok(net)) return TRAJ_E_UNSUPPORTED;
    const PackPlan pl = pack_plan(net);
    if (bytes < pl.off[11] * sizeof(float) || ((uintptr_t)packed & 15)) return TRAJ_E_ARG;
    const float* W[11] = {net->fc5_w, net->gru_q_wih, net->gru_q_whh, net->gru_sigma_wih, net->gru_sigma_whh,
                          net->fc1_w, net->fc7_w,     net->gru_s_wih, net->gru_s_whh,     net->fc3_w,
                          net->fc4_w};
    for (int i = 0; i < 11; ++i) {
        const long long n = (long long)(pl.off[i + 1] - pl.off[i]);
        hipLaunchKernelGGL(knet_pack_kernel, dim3(nblk(n, 256)), dim3(256), 0, (hipStream_t)stream, W[i], pl.N[i],
                           pl.K[i], packed + pl.off[i]);
    }
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_knet_front_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts, const traj_knet_net* net,
                        const float* packed, int B, const float* x_post, const float* u, int u_stride_b,
                        int u_stride_c, const float* y, int y_stride_b, int y_stride_c, const float* x_mean,
                        const float* x_std, const float* y_mean, const float* y_std, const float* u_mean,
                        const float* u_std, float* h_q, const float* h_sigma, float* h_s, float* m1x_prior, float* dy,
                        float* x2, void* stream) {
    if (!p || !lim || B < 0) return TRAJ_E_ARG;
    if (!knet_ok(net)) return net ? TRAJ_E_UNSUPPORTED : TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!packed || ((uintptr_t)packed & 15) || !x_post || !u || !y || !x_mean || !x_std || !y_mean || !y_std || !h_q ||
        !h_sigma || !h_s || !m1x_prior || !dy || !x2)
        return TRAJ_E_ARG;
    KP k{(float)p->Cm1, (float)p->Cm2, (float)p->Cr0, (float)p->Cr2, (float)p->Br, (float)p->Cr, (float)p->Dr,
         (float)p->Bf,  (float)p->Cf,  (float)p->Df,  (float)p->m,   (float)p->Iz, (float)p->lf, (float)p->lr,
         (float)p->maxAlpha, (float)p->vx_zero};
    hipLaunchKernelGGL(knet_front_kernel, dim3(nblk(B, KS)), dim3(KT), 0, (hipStream_t)stream, k, *lim, Ts,
                       knet_args(net, packed), B, x_post, u, u_stride_b, u_stride_c, y, y_stride_b, y_stride_c, x_mean,
                       x_std, y_mean, y_std, u_mean, u_std, h_q, h_sigma, h_s, m1x_prior, dy, x2);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

size_t traj_knet_fc2_workspace_bytes(const traj_knet_net* net, int B) {
    if (!knet_ok(net) || B < 0) return 0;
    return (size_t)(net->d_fc2h / fc2_slab(net->d_fc2h)) * (size_t)B * 32 * sizeof(float);
}

int traj_knet_fc2_f32(const traj_knet_net* net, int B, const float* x2, float* ws, size_t ws_bytes, void* stream) {
    if (B < 0) return TRAJ_E_ARG;
    if (!knet_ok(net)) return net ? TRAJ_E_UNSUPPORTED : TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!x2 || !ws || ws_bytes < traj_knet_fc2_workspace_bytes(net, B) || ((uintptr_t)x2 & 15) ||
        ((uintptr_t)net->fc2a_w & 15) || ((uintptr_t)net->fc2a_b & 15) || ((uintptr_t)net->fc2b_w & 15))
        return TRAJ_E_ARG;
    const int hs = fc2_slab(net->d_fc2h), nslab = net->d_fc2h / hs, nbb = nblk(B, F2_BT);
    return fc2_launch(net, B, x2, ws, stream);
}

int traj_knet_set_fc2_mode(int mode) {
    if (mode < 0 || mode > 2) return -1;
    return g_fc2_mode.exchange(mode);
}

int traj_knet_back_f32(const traj_knet_net* net, const float* packed, int B, const float* x2, const float* ws,
                       const float* m1x_prior, const float* dy, float* h_sigma, float* x_post, float* out,
                       int out_stride_b, int out_stride_c, float* KG_out, void* stream) {
    if (B < 0) return TRAJ_E_ARG;
    if (!knet_ok(net)) return net ? TRAJ_E_UNSUPPORTED : TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!packed || ((uintptr_t)packed & 15) || !x2 || !ws || !m1x_prior || !dy || !h_sigma || !x_post)
        return TRAJ_E_ARG;
    hipLaunchKernelGGL(knet_back_kernel, dim3(nblk(B, KS)), dim3(KT), 0, (hipStream_t)stream, knet_args(net, packed),
                       B, x2, ws, net->d_fc2h / fc2_slab(net->d_fc2h), m1x_prior, dy, h_sigma, x_post, out, out_stride_b,
                       out_stride_c, KG_out);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_knet_back_front_f32(const traj_vehicle_params* p, const traj_knet_limits* lim, float Ts,
                             const traj_knet_net* net, const float* packed, int B, const float* ws, float* out,
                             int out_stride_b, int out_stride_c, const float* u, int u_stride_b, int u_stride_c,
                             const float* y, int y_stride_b, int y_stride_c, const float* x_mean, const float* x_std,
                             const float* y_mean, const float* y_std, const float* u_mean, const float* u_std,
                             float* h_q, float* h_sigma, float* h_s, float* x_post, float* m1x_prior, float* dy,
                             float* x2, void* stream) {
    if (!p || !lim || B < 0) return TRAJ_E_ARG;
    if (!knet_ok(net)) return net ? TRAJ_E_UNSUPPORTED : TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!packed || ((uintptr_t)packed & 15) || !ws || !u || !y || !x_mean || !x_std || !y_mean || !y_std || !h_q ||
        !h_sigma || !h_s || !x_post || !m1x_prior || !dy || !x2)
        return TRAJ_E_ARG;
    KP k{(float)p->Cm1, (float)p->Cm2, (float)p->Cr0, (float)p->Cr2, (float)p->Br, (float)p->Cr, (float)p->Dr,
         (float)p->Bf,  (float)p->Cf,  (float)p->Df,  (float)p->m,   (float)p->Iz, (float)p->lf, (float)p->lr,
         (float)p->maxAlpha, (float)p->vx_zero};
    if (!out) return TRAJ_E_ARG;
    hipLaunchKernelGGL(knet_back_front_kernel, dim3(nblk(B, KS)), dim3(KT), 0, (hipStream_t)stream,
                       knet_args(net, packed), B, ws, net->d_fc2h / fc2_slab(net->d_fc2h), out, out_stride_b,
                       out_stride_c, k, *lim, Ts, u, u_stride_b, u_stride_c, y, y_stride_b, y_stride_c, x_mean, x_std,
                       y_mean, y_std, u_mean, u_std, h_q, h_sigma, h_s, x_post, m1x_prior, dy, x2);
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
