// mpc_inst.hip -- one translation unit per horizon capacity (compiled with -DTGMPC_NN=<NN>), so
// the fully unrolled instantiations of the MPC kernels build in parallel.
#include <atomic>

#include "mpc_launch.h"

#ifndef TGMPC_NN
#error "compile with -DTGMPC_NN=<capacity>"
#endif

#define TGMPC_CAT2(a, b) a##b
#define TGMPC_CAT(a, b) TGMPC_CAT2(a, b)

namespace tgmpc {

#if TGMPC_NN == 40
int launch_fused_w3_40(const KArgs& a, hipStream_t st);   // mpc_inst_w3.hip
void preload_fused_w3_40();                                // mpc_inst_w3.hip
#endif

// mode 0: MPC step, 1: QP only (A/B/g given), 2: closed-loop step (the linearization launches are
// issued by the caller, trajmpc.hip), 3: fused closed loop of a.nsteps steps (linearization inside),
// 4: MPC step with the linearization inside (one launch; the records go to the workspace's A/B/g)
int TGMPC_CAT(launch_mpc_, TGMPC_NN)(const KArgs& a, hipStream_t st, int mode) {
    constexpr int NN = TGMPC_NN;
    dim3 grid(a.B), sblock(((NN + 63) / 64) * 64);
    if (mode == 3) {
#if TGMPC_NN == 40
        {
            // HIP loads a kernel's code object at its first launch (milliseconds of host time for these): the first
            // fused launch at this capacity loads BOTH instances, so a later launch of the other one (the opt-in
            // 3-wave instance, traj_debug_fused_waves(3)) does not pay it inside its own call.  Per device.
            static std::atomic<bool> loaded[64];
            int dev = 0;
            if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 && !loaded[dev].load()) {
                hipFuncAttributes fa;
                preload_fused_w3_40();
                if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&solve_kernel<NN, true, true, false, 2>)) ==
                    hipSuccess)
                    loaded[dev].store(true);
            }
        }
        if (a.wps == 3) return launch_fused_w3_40(a, st);
#endif
#if TGMPC_NN > 64
        // capacity 80: one wave per SIMD (the default, a.wps = 1) unless the lean two-wave instance (2 waves per
        // SIMD, 4 instances per CU, opt-in) is asked for with traj_debug_fused_waves(2); any other value runs the
        // default
        if (a.wps != 2) return launch_fused<NN, 1>(a, st);
#endif
        return launch_fused<NN, 2>(a, st);
    }
    else if (mode == 2) hipLaunchKernelGGL((solve_kernel<NN, true>), grid, sblock, 0, st, a);
    else if (mode == 4) hipLaunchKernelGGL((solve_kernel<NN, false, false, true, 2, true>), grid, sblock, 0, st, a);
    else hipLaunchKernelGGL((solve_kernel<NN, false>), grid, sblock, 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace tgmpc
