// Checks the lane semantics of the DPP wave shifts used for the +-2 exchanges.
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ inline double sh(double v, int ctrl) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    if (ctrl == 0) { lo = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xf, 0xf, false); }
    else { lo = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xf, 0xf, false); }
    return __hiloint2double(hi, lo);
}
__global__ void k(double* o) {
    int t = threadIdx.x;
    double v = 100.0 + t;
    o[t] = sh(sh(v, 0), 0);
    o[64 + t] = sh(sh(v, 1), 1);
}
int main() {
    double* d; hipMalloc(&d, 128 * 8);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    double h[128]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("shl1 x2: lane0 %.0f lane1 %.0f lane15 %.0f lane16 %.0f lane61 %.0f lane62 %.0f lane63 %.0f\n", h[0], h[1], h[15], h[16], h[61], h[62], h[63]);
    printf("shr1 x2: lane0 %.0f lane1 %.0f lane2 %.0f lane16 %.0f lane17 %.0f lane63 %.0f\n", h[64], h[65], h[66], h[80], h[81], h[127]);
    return 0;
}
