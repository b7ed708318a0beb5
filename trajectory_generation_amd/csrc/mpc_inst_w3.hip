// mpc_inst_w3.hip -- the fused closed-loop kernel at capacity 40 held to 3 waves per SIMD (168 VGPRs, the compact
// LDS image of 12.8 KB: 12 one-wave workgroups per CU).  Built with the AMDGPU register-pressure trackers in the
// scheduler (-amdgpu-use-amdgpu-trackers): with the default trackers the ADMM loop spilled its constants to
// scratch at this budget.  Bit-identical to the 2-wave instance (same arithmetic, same order); trajmpc.hip picks
// it for long launches (TRAJ_FUSED_W3_MIN_STEPS).
#include "mpc_launch.h"

namespace tgmpc {

int launch_fused_w3_40(const KArgs& a, hipStream_t st) { return launch_fused<40, 3>(a, st); }

// load the instance's code object without launching it (mpc_inst.hip's first fused launch at capacity 40)
void preload_fused_w3_40() {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&solve_kernel<40, true, true, false, 3>));
}

}  // namespace tgmpc
