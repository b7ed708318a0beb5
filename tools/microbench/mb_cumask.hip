// Feasibility probe: do two streams with disjoint CU masks (hipExtStreamCreateWithCUMask) run their kernels on
// disjoint CUs of MI355X, and how do mask bits map to (XCC, SE, CU)?  Stream H gets the first NH mask bits,
// stream B the rest; a spinning kernel on each records HW_ID / XCC_ID per workgroup.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void where(unsigned* out, long long spin) {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) { out[2 * blockIdx.x] = hw; out[2 * blockIdx.x + 1] = xcc; }
}

static void key(unsigned hw, unsigned xcc, int& cu, int& simd) {
    const int c = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    simd = (hw >> 4) & 3;
    cu = ((xcc & 7) * 8 + se * 2 + sh) * 16 + c;
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("CUs %d\n", ncu);
    for (int NH : {4, 8, 16}) {
        std::vector<uint32_t> mh((ncu + 31) / 32, 0), mb((ncu + 31) / 32, 0);
        for (int i = 0; i < ncu; ++i) (i < NH ? mh : mb)[i / 32] |= 1u << (i % 32);
        hipStream_t sh, sb;
        if (hipExtStreamCreateWithCUMask(&sh, ncu, mh.data()) != hipSuccess ||
            hipExtStreamCreateWithCUMask(&sb, ncu, mb.data()) != hipSuccess) { printf("mask stream failed\n"); return 1; }
        const int GH = 4 * NH, GB = 8 * ncu;
        unsigned *dh, *db;
        (void)hipMalloc(&dh, GH * 8); (void)hipMalloc(&db, GB * 8);
        hipLaunchKernelGGL(where, dim3(GB), dim3(64), 0, sb, db, 20000LL);   // 200 us at 100 MHz
        hipLaunchKernelGGL(where, dim3(GH), dim3(64), 0, sh, dh, 5000LL);
        if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
        std::vector<unsigned> h(2 * GH), b(2 * GB);
        (void)hipMemcpy(h.data(), dh, GH * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(b.data(), db, GB * 8, hipMemcpyDeviceToHost);
        std::set<int> ch, cb, simds;
        for (int i = 0; i < GH; ++i) { int c, s; key(h[2 * i], h[2 * i + 1], c, s); ch.insert(c); simds.insert(c * 4 + s); }
        for (int i = 0; i < GB; ++i) { int c, s; key(b[2 * i], b[2 * i + 1], c, s); cb.insert(c); }
        int overlap = 0;
        for (int c : ch) overlap += cb.count(c);
        printf("NH %2d: H grid %d on %zu CUs (%zu distinct SIMDs), B grid %d on %zu CUs, overlap %d; H CUs:", NH, GH,
               ch.size(), simds.size(), GB, cb.size(), overlap);
        for (int c : ch) printf(" x%d/se%d/cu%d", c / 128, (c / 16) % 8, c % 16);
        printf("\n");
        (void)hipFree(dh); (void)hipFree(db);
        (void)hipStreamDestroy(sh); (void)hipStreamDestroy(sb);
    }
    return 0;
}
