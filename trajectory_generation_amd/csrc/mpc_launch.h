// mpc_launch.h -- the fused closed-loop launch (traj_closed_loop_run), shared by the per-capacity translation
// units: mpc_inst.hip (every capacity, 2 waves per SIMD) and mpc_inst_w3.hip (NN = 40 at 3 waves per SIMD).
#pragma once
#include "mpc_solve.h"

namespace tgmpc {

// One workgroup per resident slot (occupancy x CUs), each taking (step, instance) items from the queue; at
// least ceil(B / TRAJ_FUSED_MAX_PER_WG) workgroups.  The production instance has no diagnostics compiled in;
// a.dbg / a.dbg_items select the DIAG one, whose residency can differ -- each has its own slot count.
template <int NN, int WPS>
int launch_fused(const KArgs& a, hipStream_t st) {
    const dim3 sblock(((NN + 63) / 64) * 64);
    const bool diag = a.dbg != nullptr || a.dbg_items != nullptr;
    static int slots_per_cu[2][64] = {{0}};
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -3;
    if (!slots_per_cu[diag][dev]) {
        int nb = 0, ncu = 0;
        const hipError_t e =
            diag ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, solve_kernel<NN, true, true, true, WPS>, (int)sblock.x, 0)
                 : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, solve_kernel<NN, true, true, false, WPS>, (int)sblock.x, 0);
        if (e != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -3;
        constexpr int WAVES = (NN + 63) / 64;
        const int cap = 4 * WPS / WAVES;   // WPS waves per SIMD, 4 SIMDs, WAVES waves per workgroup
        slots_per_cu[diag][dev] = nb < 1 ? 1 : (nb > cap ? cap : nb);
        cus[dev] = ncu < 1 ? 1 : ncu;
    }
    int G = a.fused_grid > 0 ? a.fused_grid : slots_per_cu[diag][dev] * cus[dev];
    if (G > a.B) G = a.B;
    const int minG = (a.B + TRAJ_FUSED_MAX_PER_WG - 1) / TRAJ_FUSED_MAX_PER_WG;
    if (G < minG) G = minG;
    if (diag) hipLaunchKernelGGL((solve_kernel<NN, true, true, true, WPS>), dim3(G), sblock, 0, st, a);
    else hipLaunchKernelGGL((solve_kernel<NN, true, true, false, WPS>), dim3(G), sblock, 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace tgmpc
