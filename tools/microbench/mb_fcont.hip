// Microbenchmark: latency (dependent chain, 1 lane) and throughput (all lanes) of one f_cont.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../../include/trajmpc.h"
#include "../../trajectory_generation_amd/csrc/physics.h"
using namespace tgmpc;
constexpr int K = 200;
__global__ void lat(traj_vehicle_params p, double* out, long long* cyc) {
    double x[6] = {0.1, 0.5, 0.05, 1.0 + 1e-3 * threadIdx.x, 0.01, 0.2}, f[6], u[2] = {0.2, 0.05};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < K; ++k) {
        f_cont(p, x, u, f);
        for (int i = 0; i < 6; ++i) x[i] += 1e-4 * f[i];
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 6; ++i) out[(blockIdx.x * blockDim.x + threadIdx.x) * 6 + i] = x[i];
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    traj_vehicle_params p;
    p.Cm1 = .287; p.Cm2 = .0545; p.Cr0 = .0518; p.Cr2 = .00035; p.Br = 3.3852; p.Cr = 1.2691; p.Dr = .1737;
    p.Bf = 2.579; p.Cf = 1.2; p.Df = .192; p.m = .041; p.Iz = 27.8e-6; p.lf = .029; p.lr = .033; p.g = 9.81;
    p.maxAlpha = .6; p.vx_zero = .3;
    double* out; long long* cyc;
    hipMalloc(&out, 1 << 26); hipMalloc(&cyc, 1 << 20);
    for (int cfg = 0; cfg < 3; ++cfg) {
        int blocks = cfg == 0 ? 1 : (cfg == 1 ? 1024 : 8192), threads = 64;
        hipLaunchKernelGGL(lat, dim3(blocks), dim3(threads), 0, 0, p, out, cyc);
        hipDeviceSynchronize();
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        hipEventRecord(e0);
        hipLaunchKernelGGL(lat, dim3(blocks), dim3(threads), 0, 0, p, out, cyc);
        hipEventRecord(e1); hipDeviceSynchronize();
        float ms; hipEventElapsedTime(&ms, e0, e1);
        std::vector<long long> c(blocks);
        hipMemcpy(c.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
        std::sort(c.begin(), c.end());
        printf("blocks %5d x 64 lanes: %.0f cycles per dependent f_cont (median wave); kernel %.3f ms -> %.2f ns per f_cont (all lanes)\n",
               blocks, (double)c[blocks / 2] / K, ms, 1e6 * ms / ((double)blocks * threads * K));
    }
    return 0;
}
