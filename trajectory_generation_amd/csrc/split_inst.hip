// split_inst.hip -- the row-split kernel's instantiations (mpc_split.h) and their launches, in a translation unit of
// their own so that it is compiled like the other register-resident solvers (no machine-level LICM: hoisting per-lane
// values out of the sweep and ADMM loops keeps them live across the whole solve and spills).
#include <cstdint>

#include "mpc_split.h"

namespace tgmpc {

// Row-split solve for TRAJ_MAX_N < N <= TRAJ_MAX_N_SPLIT: H = 48 (n <= 96, 3 waves) or 64 (n <= 128, 4 waves) per
// instance.  sws: the caller's scratch (traj_mpc_sb_workspace_bytes), aligned up to 16 bytes here for the 16-byte P
// row loads (B split_ws_doubles(N) + 2 <= B gen_ws_doubles(N) doubles: the slack fits).
template <bool CLOSED>
static int launch_split_t(const KArgs& a, double* sws, hipStream_t st) {
    const int N = a.c.N, n = 2 * N;
    double* al = reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(sws) + 15) & ~uintptr_t(15));
    const size_t per = split_ws_doubles(N);
    if (split_h(n) == 48)
        hipLaunchKernelGGL((solve_split_kernel<48, CLOSED>), dim3(a.B), dim3(SplitCfg<48>::NT), 0, st, a, al, per);
    else
        hipLaunchKernelGGL((solve_split_kernel<64, CLOSED>), dim3(a.B), dim3(SplitCfg<64>::NT), 0, st, a, al, per);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_split_step(const KArgs& a, double* sws, hipStream_t st) { return launch_split_t<false>(a, sws, st); }
int launch_split_closed(const KArgs& a, double* sws, hipStream_t st) { return launch_split_t<true>(a, sws, st); }

}  // namespace tgmpc
