// mpc_inst.hip -- one translation unit per horizon capacity (compiled with -DTGMPC_NN=<NN>), so
// the fully unrolled instantiations of the MPC kernels build in parallel.
#include "mpc_solve.h"

#ifndef TGMPC_NN
#error "compile with -DTGMPC_NN=<capacity>"
#endif

#define TGMPC_CAT2(a, b) a##b
#define TGMPC_CAT(a, b) TGMPC_CAT2(a, b)

namespace tgmpc {

// mode 0: MPC step, 1: QP only (A/B/g given), 2: closed-loop step (the linearization launches are
// issued by the caller, trajmpc.hip), 3: fused closed loop of a.nsteps steps (linearization inside)
int TGMPC_CAT(launch_mpc_, TGMPC_NN)(const KArgs& a, hipStream_t st, int mode) {
    constexpr int NN = TGMPC_NN;
    dim3 grid(a.B), sblock(((NN + 63) / 64) * 64);
    if (mode == 3) {
        // fused: one workgroup per resident slot (occupancy x CUs), each running its instances
        // step by step; at most TRAJ_FUSED_MAX_PER_WG instances per workgroup
        static int slots_per_cu[64] = {0};
        static int cus[64] = {0};
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -3;
        if (!slots_per_cu[dev]) {
            int nb = 0, ncu = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, solve_kernel<NN, true, true>, (int)sblock.x, 0) !=
                    hipSuccess ||
                hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
                return -3;
            slots_per_cu[dev] = nb < 1 ? 1 : (nb > 8 ? 8 : nb);
            cus[dev] = ncu < 1 ? 1 : ncu;
        }
        int G = a.fused_grid > 0 ? a.fused_grid : slots_per_cu[dev] * cus[dev];
        if (G > a.B) G = a.B;
        const int minG = (a.B + TRAJ_FUSED_MAX_PER_WG - 1) / TRAJ_FUSED_MAX_PER_WG;
        if (G < minG) G = minG;
        hipLaunchKernelGGL((solve_kernel<NN, true, true>), dim3(G), sblock, 0, st, a);
    }
    else if (mode == 2) hipLaunchKernelGGL((solve_kernel<NN, true>), grid, sblock, 0, st, a);
    else hipLaunchKernelGGL((solve_kernel<NN, false>), grid, sblock, 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace tgmpc
