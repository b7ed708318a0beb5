// Microbenchmark: cost of one dense register mat-vec y = K v (K row per lane, NN doubles) with the
// vector broadcast through LDS vs v_readlane, and of a +-2 lane exchange through LDS vs DPP.
// One wave per workgroup, many workgroups; prints cycles per iteration (median over waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int NN = 40;
constexpr int ITERS = 2000;

__device__ inline double shfl_dpp_shr1(double v) {   // value of lane t-1 (0 for lane 0)
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ inline double shfl_dpp_shl1(double v) {   // value of lane t+1
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xf, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ inline double readlane_d(double v, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ __launch_bounds__(64) void kmul_bench(const double* Kin, double* out, long long* cyc) {
    __shared__ double buf[4][NN + 8];
    const int t = threadIdx.x;
    double K[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) K[j] = Kin[(t % NN) * NN + j] * (t < NN ? 1.0 : 0.0);
    double v = 1.0 + 1e-3 * t;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        double y;
        if (MODE == 0) {            // LDS broadcast (write, barrier, 20 x ds_read_b128)
            double* b = buf[it & 3];
            if (t < NN) b[t] = v;
            __syncthreads();
            double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
            for (int j = 0; j < NN; j += 4) {
                s0 = fma(K[j], b[j], s0); s1 = fma(K[j + 1], b[j + 1], s1);
                s2 = fma(K[j + 2], b[j + 2], s2); s3 = fma(K[j + 3], b[j + 3], s3);
            }
            y = (s0 + s1) + (s2 + s3);
        } else if (MODE == 1) {     // v_readlane broadcast
            double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll
            for (int j = 0; j < NN; j += 4) {
                s0 = fma(K[j], readlane_d(v, j), s0); s1 = fma(K[j + 1], readlane_d(v, j + 1), s1);
                s2 = fma(K[j + 2], readlane_d(v, j + 2), s2); s3 = fma(K[j + 3], readlane_d(v, j + 3), s3);
            }
            y = (s0 + s1) + (s2 + s3);
        } else if (MODE == 2) {     // +-2 exchange through LDS (x2: one up, one down)
            double* b = buf[it & 3];
            if (t < NN) b[t + 2] = v;
            __syncthreads();
            double up = b[t + 4 < NN + 8 ? t + 4 : 0];
            double* b2 = buf[(it + 1) & 3];
            if (t < NN) b2[t + 2] = up;
            __syncthreads();
            y = b2[t] + 0.5 * v;
        } else if (MODE == 4) {     // LDS broadcast, 8 accumulation chains
            double* b = buf[it & 3];
            if (t < NN) b[t] = v;
            __syncthreads();
            double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NN; ++j) s[j & 7] = fma(K[j], b[j], s[j & 7]);
            y = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        } else if (MODE == 5) {     // register-only: 40 FMAs (8 chains), v from lane itself
            double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NN; ++j) s[j & 7] = fma(K[j], v, s[j & 7]);
            y = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        } else if (MODE == 6) {     // LDS broadcast, wave barrier only (single-wave workgroup)
            double* b = buf[it & 3];
            if (t < NN) b[t] = v;
            __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
            __builtin_amdgcn_wave_barrier();
            double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int j = 0; j < NN; ++j) s[j & 7] = fma(K[j], b[j], s[j & 7]);
            y = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        } else if (MODE == 3) {     // +-2 exchange through DPP wave shifts
            double up = shfl_dpp_shl1(shfl_dpp_shl1(v));
            double dn = shfl_dpp_shr1(shfl_dpp_shr1(up));
            y = dn + 0.5 * v;
        } else { y = v; }
        v = 0.999 * y + 1e-3;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + t] = v;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, int nblk, double* dK, double* dout, long long* dcyc) {
    hipLaunchKernelGGL(kmul_bench<MODE>, dim3(nblk), dim3(64), 0, 0, dK, dout, dcyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kmul_bench<MODE>, dim3(nblk), dim3(64), 0, 0, dK, dout, dcyc);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c(nblk);
    hipMemcpy(c.data(), dcyc, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    printf("%-28s blocks %5d: %8.1f cycles/iter (median wave), kernel %.3f ms -> %.1f ns per wave-iter\n", name, nblk,
           (double)c[nblk / 2] / ITERS, ms, 1e6 * ms / ((double)nblk * ITERS));
}

int main() {
    double *dK, *dout; long long* dcyc;
    std::vector<double> K(NN * NN);
    for (int i = 0; i < NN; ++i) for (int j = 0; j < NN; ++j) K[i * NN + j] = (i == j ? 0.5 : 0.01 / (1 + std::abs(i - j)));
    hipMalloc(&dK, K.size() * 8); hipMalloc(&dout, 65536 * 64 * 8); hipMalloc(&dcyc, 65536 * 8);
    hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
    for (int nb : {1024, 4096, 16384}) {
        run<0>("kmul LDS broadcast", nb, dK, dout, dcyc);
        run<1>("kmul readlane", nb, dK, dout, dcyc);
        run<2>("exchange +-2 LDS", nb, dK, dout, dcyc);
        run<3>("exchange +-2 DPP", nb, dK, dout, dcyc);
        run<4>("kmul LDS 8 chains", nb, dK, dout, dcyc);
        run<5>("kmul regs only 8 chains", nb, dK, dout, dcyc);
        run<6>("kmul LDS wavebarrier 8ch", nb, dK, dout, dcyc);
    }
    return 0;
}
