// Microbenchmark: latency of one ADMM iteration of solve_kernel (mpc_solve.h, phase PH_ADMM) for
// NN = 40 variables on one wave -- the same helpers (DPP +-2 exchanges, LDS broadcast + register
// mat-vec with K^{-1} rows, projections) -- and variants of its LDS broadcast.  Prints cycles per
// iteration (median wave) at 1 and 2 waves per SIMD, and checks that the variants that must be
// bit-identical are.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../trajectory_generation_amd/csrc/mpc_common.h"

using namespace tgmpc;
constexpr int NN = 40;

// V 0: bcast = ds_write + __syncthreads (current); 1: ds_write + compiler fence only (one wave: LDS
// executes a wave's DS instructions in order); 2: as 1 with one DPP per exchange (cost probe, not
// equivalent); 3: Kmul only; 4: everything but Kmul
template <int V>
__global__ __launch_bounds__(64) void admm_bench(const double* Kin, double* out, long long* cyc, int iters) {
    __shared__ __attribute__((aligned(16))) double s_ex[4 * NN + 8];
    const int t = threadIdx.x;
    const int n = NN;
    const bool own = t < n;
    const bool has_prev = (t >> 1) > 0;
    for (int i = t; i < 4 * NN + 8; i += 64) s_ex[i] = 0.0;
    __syncthreads();
    double Krow[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) Krow[j] = own ? Kin[t * NN + j] : 0.0;
    const double a_b = 0.9 + 0.001 * t, a_r = 0.8 + 0.002 * t, a_rm = has_prev ? 0.7 : 0.0, a_rp = 0.75;
    const double rb = 0.1, rr = 0.12, rb_inv = 1.0 / rb, rr_inv = 1.0 / rr, sig = 1e-6, alpha = 1.6;
    const double slb = -0.5, sub = 0.5, slr = -0.05, sur = 0.05, qi = 0.01 * (t - 20);
    int xb = 0;
    auto exch = [&](double v, int delta) -> double {
        const double vm = own ? v : 0.0;
        double r;
        if (V == 2) r = (delta > 0) ? dpp_d<0x130>(vm) : dpp_d<0x138>(vm);
        else r = (delta > 0) ? lane_up2(vm) : lane_dn2(vm);
        return own ? r : 0.0;
    };
    auto Kmul = [&](double v) -> double {
        double* buf = s_ex + (xb & 3) * NN;
        xb++;
        if (own) buf[t] = v;
        if (V == 1 || V == 2) {
            __builtin_amdgcn_wave_barrier();
            asm volatile("" ::: "memory");
        } else {
            __syncthreads();
        }
        double vb[NN];
        if (V == 6) {
#pragma unroll
            for (int j = 0; j < NN; ++j) vb[j] = v + j;
        } else {
            lds_load_all<NN>(buf, vb);
        }
        if (V == 5) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < NN; j += 8) s += vb[j];
            return own ? s : 0.0;
        }
        if (V == 7) {
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j < NN; ++j) s4[j & 3] = fma(Krow[j], vb[j], s4[j & 3]);
            return own ? (s4[0] + s4[1]) + (s4[2] + s4[3]) : 0.0;
        }
        double sa[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < NN; ++j) sa[j & 7] = fma(Krow[j], vb[j], sa[j & 7]);
        return own ? ((sa[0] + sa[1]) + (sa[2] + sa[3])) + ((sa[4] + sa[5]) + (sa[6] + sa[7])) : 0.0;
    };
    auto Ax = [&](double v, double& zb_, double& zr_) {
        double vdn = exch(v, -2);
        zb_ = a_b * v;
        zr_ = a_r * v - a_rm * vdn;
    };
    auto ATw = [&](double wb, double wr) -> double {
        double wr_up = exch(wr, +2);
        return a_b * wb + a_r * wr - a_rp * wr_up;
    };
    double x = 0.0, zb = 0.0, zr = 0.0, yb = 0.0, yr = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (V == 3 || V == 5 || V == 6) {
            x = 0.5 * Kmul(x + qi) + 0.001;
            continue;
        }
        if (V == 7) {
            const double oma = 1.0 - alpha;
            const double wb = fma(rb, zb, -yb), wr = fma(rr, zr, -yr);
            const double wr_up = exch(wr, +2);
            const double atw = fma(a_b, wb, fma(a_r, wr, -a_rp * wr_up));
            const double xt = Kmul(fma(sig, x, atw - qi));
            const double vdn = exch(xt, -2);
            const double ztb = a_b * xt, ztr = fma(a_r, xt, -a_rm * vdn);
            const double xn = fma(alpha, xt, oma * x);
            const double zrb = fma(alpha, ztb, oma * zb), zrr = fma(alpha, ztr, oma * zr);
            const double nzb = clampd(fma(rb_inv, yb, zrb), slb, sub), nzr = clampd(fma(rr_inv, yr, zrr), slr, sur);
            yb = fma(rb, zrb - nzb, yb);
            yr = fma(rr, zrr - nzr, yr);
            x = xn;
            zb = nzb;
            zr = nzr;
            continue;
        }
        double rhs = sig * x - qi + ATw(rb * zb - yb, rr * zr - yr);
        double xt = (V == 4) ? 0.5 * rhs : Kmul(rhs);
        double ztb, ztr;
        Ax(xt, ztb, ztr);
        double xn = alpha * xt + (1.0 - alpha) * x;
        double zrb = alpha * ztb + (1.0 - alpha) * zb;
        double zrr = alpha * ztr + (1.0 - alpha) * zr;
        double vb = zrb + rb_inv * yb, vr = zrr + rr_inv * yr;
        double nzb = clampd(vb, slb, sub), nzr = clampd(vr, slr, sur);
        yb = yb + rb * (zrb - nzb);
        yr = yr + rr * (zrr - nzr);
        x = xn;
        zb = nzb;
        zr = nzr;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + t] = x + zb + zr + yb + yr;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static double run(const char* name, int nblk, int iters, const double* dK, double* dout, long long* dcyc,
                  std::vector<double>* res) {
    hipLaunchKernelGGL(admm_bench<V>, dim3(nblk), dim3(64), 0, 0, dK, dout, dcyc, iters);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(admm_bench<V>, dim3(nblk), dim3(64), 0, 0, dK, dout, dcyc, iters);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c(nblk);
    hipMemcpy(c.data(), dcyc, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    if (res) {
        res->resize((size_t)nblk * 64);
        hipMemcpy(res->data(), dout, res->size() * 8, hipMemcpyDeviceToHost);
    }
    std::sort(c.begin(), c.end());
    const double cpi = (double)c[nblk / 2] / iters;
    printf("%-34s blocks %5d: %7.1f cycles/iter (median wave), %.1f ns/iter wall\n", name, nblk, cpi,
           1e6 * ms / iters);
    return cpi;
}

int main() {
    double *dK, *dout;
    long long* dcyc;
    std::vector<double> K(NN * NN);
    for (int i = 0; i < NN; ++i)
        for (int j = 0; j < NN; ++j) K[i * NN + j] = (i == j ? 0.5 : 0.01 / (1 + std::abs(i - j)));
    hipMalloc(&dK, K.size() * 8);
    hipMalloc(&dout, 8192 * 64 * 8);
    hipMalloc(&dcyc, 8192 * 8);
    hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
    const int iters = 4000;
    for (int nb : {1024, 2048}) {
        std::vector<double> r0, r1;
        run<0>("admm iteration (syncthreads)", nb, iters, dK, dout, dcyc, &r0);
        run<1>("admm iteration (no LDS wait)", nb, iters, dK, dout, dcyc, &r1);
        run<2>("  + one DPP per exchange (probe)", nb, iters, dK, dout, dcyc, nullptr);
        run<3>("Kmul only", nb, iters, dK, dout, dcyc, nullptr);
        run<4>("everything but Kmul", nb, iters, dK, dout, dcyc, nullptr);
        run<5>("Kmul LDS part only", nb, iters, dK, dout, dcyc, nullptr);
        run<6>("Kmul FMA part only", nb, iters, dK, dout, dcyc, nullptr);
        std::vector<double> r7;
        run<7>("contracted + 4 chains", nb, iters, dK, dout, dcyc, &r7);
        double md = 0;
        for (size_t i = 0; i < r0.size(); ++i) md = std::max(md, std::abs(r0[i] - r7[i]) / (1e-300 + std::abs(r0[i])));
        printf("  variant 7 vs 0: max rel diff %.3e\n", md);
        size_t ndiff = 0;
        for (size_t i = 0; i < r0.size(); ++i) ndiff += (r0[i] != r1[i]);
        printf("  variant 1 vs 0: %zu of %zu outputs differ\n", ndiff, r0.size());
    }
    return 0;
}
