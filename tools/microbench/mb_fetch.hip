// Microbenchmark: what rocprofv3's FETCH_SIZE counts on gfx950 for the read patterns of the fused MPC kernel,
// against known bytes -- to decide whether the guide's x2 correction (established for wide coalesced 16 B/lane
// streams, MI355X_MICROARCH.md "HBM") applies to solve_kernel's small reads.
//
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/mb_fetch.hip -o mb_fetch
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- ./mb_fetch      (then tools/mb_fetch_report.py)
//
// Every kernel reads its own region of a 3 GiB buffer once (no reuse: the 256 MB MALL and the L2s cannot
// hold a region between kernels), 64 MiB of cache lines per kernel:
//   k_stream16   16 B per lane, coalesced (global_load_dwordx4): useful bytes = line bytes
//   k_scatter8   one 8-B load per lane, each to its own 128-B line (stride 128 B): useful 8 B per line
//   k_scatter8c  the same with coherent (sc1) loads -- the fused kernel's hand-off reads (ld_coh)
//   k_run8       one lane per wave reads a run of 21 consecutive doubles (the vref row of an instance) with
//                8-B loads, runs 256 B apart: useful 168 B per 256 B of lines
// The per-dispatch FETCH_SIZE (KiB) is printed beside these numbers by tools/mb_fetch_report.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr size_t REGION = 64ull << 20;   // bytes of cache lines each kernel touches

__global__ void k_stream16(const double2* __restrict__ p, double* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double2 v = p[i];
    if (v.x == 12345.0) out[0] = v.y;   // never true: keeps the load
}
__global__ void k_scatter8(const double* __restrict__ p, double* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double v = p[i * 16];   // 128-B stride
    if (v == 12345.0) out[0] = v;
}
__global__ void k_scatter8c(const double* __restrict__ p, double* out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const double v = __hip_atomic_load(const_cast<double*>(p) + i * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v == 12345.0) out[0] = v;
}
__global__ void k_run8(const double* __restrict__ p, double* out) {
    // one lane per wave; run r = wave index; 21 doubles at 256-B spacing of runs
    const size_t r = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / 64;
    if ((threadIdx.x & 63) != 0) return;
    const double* q = p + r * 32;
    double s = 0.0;
    for (int k = 0; k < 21; ++k) s += q[k];
    if (s == 12345.0) out[0] = s;
}

int main() {
    const size_t total = 4 * REGION + (64ull << 20);
    char* buf = nullptr;
    double* out = nullptr;
    if (hipMalloc(&buf, total) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    if (hipMemset(buf, 1, total) != hipSuccess) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const int bs = 256;
    // k_stream16: REGION / 16 lanes
    hipLaunchKernelGGL(k_stream16, dim3(REGION / 16 / bs), dim3(bs), 0, 0, (const double2*)(buf + 0 * REGION), out);
    // k_scatter8(c): one lane per 128-B line
    hipLaunchKernelGGL(k_scatter8, dim3(REGION / 128 / bs), dim3(bs), 0, 0, (const double*)(buf + 1 * REGION), out);
    hipLaunchKernelGGL(k_scatter8c, dim3(REGION / 128 / bs), dim3(bs), 0, 0, (const double*)(buf + 2 * REGION), out);
    // k_run8: one run per 256 B -> REGION / 256 runs = waves
    hipLaunchKernelGGL(k_run8, dim3(REGION / 256 * 64 / bs), dim3(bs), 0, 0, (const double*)(buf + 3 * REGION), out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    const double mib = REGION / 1048576.0;
    printf("{\"region_bytes\": %zu, \"kernels\": {\n", REGION);
    printf(" \"k_stream16\": {\"useful_bytes\": %zu, \"line_bytes\": %zu},\n", REGION, REGION);
    printf(" \"k_scatter8\": {\"useful_bytes\": %zu, \"line_bytes\": %zu},\n", REGION / 16, REGION);
    printf(" \"k_scatter8c\": {\"useful_bytes\": %zu, \"line_bytes\": %zu},\n", REGION / 16, REGION);
    printf(" \"k_run8\": {\"useful_bytes\": %zu, \"line_bytes\": %zu}}, \"region_mib\": %.0f}\n", REGION / 256 * 168,
           REGION / 256 * 192, mib);
    hipFree(buf);
    hipFree(out);
    return 0;
}
