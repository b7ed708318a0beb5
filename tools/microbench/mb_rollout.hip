// Microbenchmark: block_linearize (the fused kernel's rollout + central-difference linearization, N = 20,
// 64 lanes per instance) in isolation -- cycles of the rollout loop and of the assembly pass (median
// workgroup), at 1 and 2 workgroups per SIMD, for instruction-count work on the rollout (rocprofv3 --pmc
// SQ_INSTS_VALU ... over this binary gives VALU instructions per instance: SQ_WAVES = instances).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off [-DTGMPC_FASTMATH=1] -o mb_rollout.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#include "../../trajectory_generation_amd/csrc/mpc_linearize.h"

using namespace tgmpc;
constexpr int N = 20;

__global__ __launch_bounds__(64) void roll(VP p, double Ts, double* out, long long* dbg) {
    __shared__ double xs[6], us[2];
    __shared__ __attribute__((aligned(16))) double rec[LREC * N];
    const int t = threadIdx.x, b = blockIdx.x;
    if (t == 0) {
        const double h = 1e-3 * (b % 997);
        xs[0] = 0.1 + h; xs[1] = -0.2 + h; xs[2] = 0.3 - 2 * h; xs[3] = 1.0 + h; xs[4] = 0.02 - 0.1 * h;
        xs[5] = 0.3 - 0.5 * h;
        us[0] = 0.2 + 0.1 * h; us[1] = 0.05 - 0.2 * h;
    }
    __syncthreads();
    long long* d = dbg + (size_t)b * 32;
    if (t == 0) d[0] = __builtin_amdgcn_s_memtime();
    block_linearize<64>(t, p, N, Ts, xs, us, rec, d);
    if (t == 0) d[1] = __builtin_amdgcn_s_memtime();
    for (int i = t; i < LREC * N; i += 64) out[(size_t)b * LREC * N + i] = rec[i];
}

int main() {
    traj_vehicle_params p;
    p.Cm1 = .287; p.Cm2 = .0545; p.Cr0 = .0518; p.Cr2 = .00035; p.Br = 3.3852; p.Cr = 1.2691; p.Dr = .1737;
    p.Bf = 2.579; p.Cf = 1.2; p.Df = .192; p.m = .041; p.Iz = 27.8e-6; p.lf = .029; p.lr = .033; p.g = 9.81;
    p.maxAlpha = .6; p.vx_zero = .3;
    const int maxb = 8192;
    double* out; long long* dbg;
    hipMalloc(&out, (size_t)maxb * LREC * N * 8);
    hipMalloc(&dbg, (size_t)maxb * 32 * 8);
    std::vector<long long> h((size_t)maxb * 32);
    std::vector<double> ho((size_t)LREC * N);
    for (int rep = 0; rep < 2; ++rep)
        for (int blocks : {1024, 2048, 8192}) {
            hipMemset(dbg, 0, (size_t)maxb * 32 * 8);
            hipLaunchKernelGGL(roll, dim3(blocks), dim3(64), 0, 0, p, 0.05, out, dbg);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), dbg, (size_t)blocks * 32 * 8, hipMemcpyDeviceToHost);
            std::vector<long long> tot, rol;
            for (int b = 0; b < blocks; ++b) {
                tot.push_back(h[b * 32 + 1] - h[b * 32]);
                rol.push_back(h[b * 32 + 20] - h[b * 32]);
            }
            std::sort(tot.begin(), tot.end());
            std::sort(rol.begin(), rol.end());
            if (rep) printf("blocks %5d  rollout median %7lld  total median %7lld  (assembly %lld) cycles\n", blocks,
                            rol[blocks / 2], tot[blocks / 2], tot[blocks / 2] - rol[blocks / 2]);
        }
    hipMemcpy(ho.data(), out, ho.size() * 8, hipMemcpyDeviceToHost);
    double cs = 0;
    for (double v : ho) cs += v;
    printf("checksum %.17g\n", cs);
    return 0;
}
