// mpc_inst.hip -- one translation unit per horizon capacity (compiled with -DTGMPC_NN=<NN>), so
// the fully unrolled instantiations of mpc_step_kernel build in parallel.
#include "mpc_kernel.h"

#ifndef TGMPC_NN
#error "compile with -DTGMPC_NN=<capacity>"
#endif

#define TGMPC_CAT2(a, b) a##b
#define TGMPC_CAT(a, b) TGMPC_CAT2(a, b)

namespace tgmpc {

// mode 0: fused step (linearize + QP), 1: QP only (A/B/g given), 2: closed-loop step
int TGMPC_CAT(launch_mpc_, TGMPC_NN)(const KArgs& a, hipStream_t st, int mode) {
    constexpr int NN = TGMPC_NN;
    dim3 grid(a.B), block(((NN + 63) / 64) * 64);
    if (mode == 0) hipLaunchKernelGGL((mpc_step_kernel<NN, true, false>), grid, block, 0, st, a);
    else if (mode == 1) hipLaunchKernelGGL((mpc_step_kernel<NN, false, false>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((mpc_step_kernel<NN, true, true>), grid, block, 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace tgmpc
