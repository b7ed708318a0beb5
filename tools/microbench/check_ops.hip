// GPU check of mpc_common.h's shortcut arithmetic against the compiler's own lowering, bit for bit:
//   sqrt_n(x) vs sqrt(x), rcp_n(b) vs 1.0 / b, rcp_n(sqrt_n(x)) vs 1.0 / sqrt(x)  for x in [1e-4, 1e4] (the Ruiz
//   arguments, limit_scaling's range) and over wide normal ranges; cdiv(d, c, 1 / c) vs d / c for c = 2e-5, 1e-6, 40.
// Prints mismatch counts per case; exit status 1 if any case inside its documented range mismatches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o check_ops.bin check_ops.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

#include "../../trajectory_generation_amd/csrc/mpc_common.h"

using namespace tgmpc;

__device__ unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
// x = 10^u for u uniform in [lo, hi] (a log-uniform draw), with random low mantissa bits
__device__ double draw(unsigned long long i, double lo, double hi) {
    const unsigned long long r = mix(i);
    const double u = lo + (hi - lo) * ((r >> 11) * 0x1p-53);
    double x = exp10(u);
    unsigned long long bits;
    memcpy(&bits, &x, 8);
    bits ^= mix(i + 7) & 0xFFFFFull;
    memcpy(&x, &bits, 8);
    return x;
}
__global__ void check(int cs, double lo, double hi, unsigned long long n, unsigned long long* bad) {
    unsigned long long nb = 0;
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const double x = draw(i + (unsigned long long)cs * 0x100000000ull, lo, hi);
        double a, b;
        if (cs == 0) { a = sqrt_n(x); b = sqrt(x); }
        else if (cs == 1) { a = rcp_n(x); b = 1.0 / x; }
        else if (cs == 2) { a = rcp_n(sqrt_n(x)); b = 1.0 / sqrt(x); }
        else {
            const double c = cs == 3 ? 2.0 * 1e-5 : (cs == 4 ? 1e-6 : 40.0);
            const double d = (mix(i * 3 + 1) & 1) ? x : -x;
            a = cdiv(d, c, 1.0 / c);
            b = d / c;
        }
        unsigned long long ua, ub;
        memcpy(&ua, &a, 8);
        memcpy(&ub, &b, 8);
        nb += ua != ub;
    }
    atomicAdd(bad, nb);
}
int main() {
    struct Case { int cs; double lo, hi; const char* what; bool must; };
    const Case cases[] = {
        {0, -4, 4, "sqrt_n vs sqrt, x in [1e-4, 1e4]", true},
        {0, -300, 300, "sqrt_n vs sqrt, x in [1e-300, 1e300] (info)", false},
        {1, -2, 2, "rcp_n vs 1/x, x in [1e-2, 1e2]", true},
        {1, -4, 4, "rcp_n vs 1/x, x in [1e-4, 1e4]", true},
        {1, -250, 250, "rcp_n vs 1/x, x in [1e-250, 1e250] (info)", false},
        {2, -4, 4, "rcp_n(sqrt_n(x)) vs 1/sqrt(x), x in [1e-4, 1e4]", true},
        {3, -280, 10, "cdiv(d, 2e-5) vs d / 2e-5, |d| in [1e-280, 1e10]", true},
        {4, -280, 10, "cdiv(d, 1e-6) vs d / 1e-6, |d| in [1e-280, 1e10]", true},
        {5, -280, 10, "cdiv(d, 40) vs d / 40, |d| in [1e-280, 1e10]", true},
    };
    unsigned long long* bad;
    if (hipMalloc(&bad, 8) != hipSuccess) return 2;
    const unsigned long long n = 1ull << 28;
    int fail = 0;
    for (const Case& c : cases) {
        unsigned long long h = 0;
        if (hipMemcpy(bad, &h, 8, hipMemcpyHostToDevice) != hipSuccess) return 2;
        hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, 0, c.cs, c.lo, c.hi, n, bad);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        if (hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        printf("%-58s %llu mismatches of %llu\n", c.what, h, n);
        if (c.must && h) fail = 1;
    }
    printf(fail ? "CHECK FAILED\n" : "CHECK OK\n");
    return fail;
}
