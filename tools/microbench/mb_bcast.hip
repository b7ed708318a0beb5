// Microbenchmark: broadcast of a 40-double vector to every lane for a register mat-vec
// (the ADMM K^-1 v step of solve_kernel) at the solve kernel's occupancy (8 single-wave
// workgroups per CU, forced with 19 KB of LDS each): LDS ds_read_b128 broadcast vs v_readlane
// vs a mix.  Prints cycles per iteration (median wave) and ns per wave-iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstdlib>

constexpr int NN = 40;
constexpr int ITERS = 2000;

__device__ inline double readlane_d(double v, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

template <int NRL>   // first NRL vector entries by readlane, the rest by LDS broadcast
__global__ __launch_bounds__(64) void bc_bench(const double* Kin, double* out, long long* cyc) {
    extern __shared__ double pad[];   // 19 KB: 8 workgroups per CU, as solve_kernel
    double* buf = pad;
    const int t = threadIdx.x;
    double K[NN];
#pragma unroll
    for (int j = 0; j < NN; ++j) K[j] = Kin[(t % NN) * NN + j] * (t < NN ? 1.0 : 0.0);
    double v = 1.0 + 1e-3 * t;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITERS; ++it) {
        double* b = buf + (it & 3) * 48;
        if (NRL < NN) {
            if (t < NN) b[t] = v;
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
        }
        double s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < NN; ++j) {
            const double vj = (j < NRL) ? readlane_d(v, j) : b[j];
            s[j & 7] = fma(K[j], vj, s[j & 7]);
        }
        double y = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        v = 0.999 * y + 1e-3;
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + t] = v + pad[1000 + t];
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NRL>
void run(int nblk, double* dK, double* dout, long long* dcyc) {
    const size_t lds = getenv("MB_LDS") ? atoi(getenv("MB_LDS")) : 19072;
    hipLaunchKernelGGL(bc_bench<NRL>, dim3(nblk), dim3(64), lds, 0, dK, dout, dcyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(bc_bench<NRL>, dim3(nblk), dim3(64), lds, 0, dK, dout, dcyc);
    hipEventRecord(e1);
    hipDeviceSynchronize();
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c(nblk);
    hipMemcpy(c.data(), dcyc, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    printf("readlane %2d / LDS %2d  blocks %5d: %8.1f cycles/iter (median wave), %.2f ns per wave-iter\n", NRL, NN - NRL,
           nblk, (double)c[nblk / 2] / ITERS, 1e6 * ms / ((double)nblk * ITERS));
}

int main() {
    double *dK, *dout; long long* dcyc;
    std::vector<double> K(NN * NN);
    for (int i = 0; i < NN; ++i) for (int j = 0; j < NN; ++j) K[i * NN + j] = (i == j ? 0.5 : 0.01 / (1 + std::abs(i - j)));
    hipMalloc(&dK, K.size() * 8); hipMalloc(&dout, 65536 * 64 * 8); hipMalloc(&dcyc, 65536 * 8);
    hipMemcpy(dK, K.data(), K.size() * 8, hipMemcpyHostToDevice);
    for (int nb : {2048, 8192}) {
        run<0>(nb, dK, dout, dcyc);
        run<8>(nb, dK, dout, dcyc);
        run<16>(nb, dK, dout, dcyc);
        run<24>(nb, dK, dout, dcyc);
        run<32>(nb, dK, dout, dcyc);
        run<40>(nb, dK, dout, dcyc);
    }
    return 0;
}
