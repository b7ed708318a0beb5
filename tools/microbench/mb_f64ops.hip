// Microbenchmark: cycle costs of the f64 building blocks the MPC solve is made of, one wave per
// workgroup, at 1 and 2 waves per SIMD (grid = 256 or 512 workgroups of 64 threads on 256 CUs x 4 SIMDs:
// the runtime spreads them, so "1 wave" here means most SIMDs hold one wave, "2" two waves).
//   0 dep FMA      one dependent v_fma_f64 chain (latency per fma)
//   1 ind FMA x4   four independent chains (issue rate of one wave)
//   2 ind FMA x8   eight independent chains
//   3 MFMA dep     v_mfma_f64_16x16x4f64 on one accumulator (dependent latency)
//   4 MFMA ind x4  four accumulators (issue rate)
//   5 rcp_nr dep   v_rcp_f64 + 2 Newton steps, dependent (the sweep's 1 / d)
//   6 LDS bcast    ds_write_b64, __syncthreads, ds_read_b64 of another lane's value, dependent
//   7 DPP up2      two wave_shl:1 moves of a double (lane_up2), dependent
//   8 MFMA ind x4 + FMA x4 interleaved (do the pipes overlap within one wave?)
// Prints cycles per operation (median wave).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../trajectory_generation_amd/csrc/mpc_common.h"

using namespace tgmpc;
typedef double d4 __attribute__((ext_vector_type(4)));

template <int V>
__global__ __launch_bounds__(64) void ops(double* out, long long* cyc, int reps) {
    __shared__ double sh[128];
    const int t = threadIdx.x;
    double a = 1.0 + 1e-9 * t, b = 0.999999, c = 1e-7 * t;
    double s0 = a, s1 = a + 1, s2 = a + 2, s3 = a + 3, s4 = a + 4, s5 = a + 5, s6 = a + 6, s7 = a + 7;
    d4 acc0 = {0, 0, 0, 0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    sh[t] = a;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma nounroll
    for (int r = 0; r < reps; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if constexpr (V == 0) {
                s0 = fma3(s0, b, c);
            } else if constexpr (V == 1) {
                s0 = fma3(s0, b, c); s1 = fma3(s1, b, c); s2 = fma3(s2, b, c); s3 = fma3(s3, b, c);
            } else if constexpr (V == 2) {
                s0 = fma3(s0, b, c); s1 = fma3(s1, b, c); s2 = fma3(s2, b, c); s3 = fma3(s3, b, c);
                s4 = fma3(s4, b, c); s5 = fma3(s5, b, c); s6 = fma3(s6, b, c); s7 = fma3(s7, b, c);
            } else if constexpr (V == 3) {
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
            } else if constexpr (V == 4) {
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, c, acc1, 0, 0, 0);
                acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, c, acc2, 0, 0, 0);
                acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(c, a, acc3, 0, 0, 0);
            } else if constexpr (V == 5) {
                s0 = rcp_nr(s0 + 1.0);
            } else if constexpr (V == 6) {
                sh[t] = s0;
                __syncthreads();
                s0 = sh[(t + 1) & 63] * b;
                __syncthreads();
            } else if constexpr (V == 7) {
                s0 = lane_up2(s0) + c;
            } else if constexpr (V == 8) {
                acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc0, 0, 0, 0);
                s0 = fma3(s0, b, c); s1 = fma3(s1, b, c); s2 = fma3(s2, b, c); s3 = fma3(s3, b, c);
                acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, c, acc1, 0, 0, 0);
                s4 = fma3(s4, b, c); s5 = fma3(s5, b, c); s6 = fma3(s6, b, c); s7 = fma3(s7, b, c);
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double r = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + acc0[0] + acc1[1] + acc2[2] + acc3[3];
    out[blockIdx.x * 64 + t] = r;
    if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V>
static void run(const char* name, int nblk, int ops_per_iter) {
    const int reps = 2000;
    double* dout;
    long long* dcyc;
    hipMalloc(&dout, nblk * 64 * sizeof(double));
    hipMalloc(&dcyc, nblk * sizeof(long long));
    hipLaunchKernelGGL(ops<V>, dim3(nblk), dim3(64), 0, 0, dout, dcyc, 10);
    hipLaunchKernelGGL(ops<V>, dim3(nblk), dim3(64), 0, 0, dout, dcyc, reps);
    hipDeviceSynchronize();
    std::vector<long long> c(nblk);
    hipMemcpy(c.data(), dcyc, nblk * sizeof(long long), hipMemcpyDeviceToHost);
    std::sort(c.begin(), c.end());
    const double per = (double)c[nblk / 2] / (reps * 16.0 * ops_per_iter);
    printf("%-28s blocks %4d: %7.2f cycles per op\n", name, nblk, per);
    hipFree(dout);
    hipFree(dcyc);
}

int main() {
    for (int nb : {256 * 4, 256 * 8}) {
        run<0>("dep FMA", nb, 1);
        run<1>("ind FMA x4", nb, 4);
        run<2>("ind FMA x8", nb, 8);
        run<3>("MFMA f64 dep", nb, 1);
        run<4>("MFMA f64 ind x4", nb, 4);
        run<5>("rcp_nr dep", nb, 1);
        run<6>("LDS bcast round trip", nb, 1);
        run<7>("DPP up2 + add dep", nb, 1);
        run<8>("MFMA x2 + FMA x8 (per iter)", nb, 1);
    }
    return 0;
}
