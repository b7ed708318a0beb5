// split_inst.hip -- the row-split kernel's instantiations (mpc_split.h) and their launches, in a translation unit of
// their own so that it is compiled like the other register-resident solvers (no machine-level LICM: hoisting per-lane
// values out of the sweep and ADMM loops keeps them live across the whole solve and spills).
#include <cstdint>

#include "mpc_split.h"

namespace tgmpc {

// sws: the caller's scratch (traj_mpc_sb_workspace_bytes), aligned up to 16 bytes here for the 16-byte P row loads
// (B split_ws_doubles(N) + 2 <= B gen_ws_doubles(N) doubles: the slack fits)
static double* align16(double* p) {
    return reinterpret_cast<double*>((reinterpret_cast<uintptr_t>(p) + 15) & ~uintptr_t(15));
}

// Row-split solve for one launch of B instances (the step, the QP, one closed-loop step): H = 40 (n <= 80), 48
// (n <= 96) or 64 (n <= 128), one workgroup of 32 rows per wave per instance
// (INLIN: the step with the linearization in the workgroup, one launch per call)
template <int H, bool CLOSED, bool INLIN>
static int launch_one(const KArgs& a, double* al, size_t per, hipStream_t st) {
    hipLaunchKernelGGL((solve_split_kernel<H, CLOSED, false, INLIN>), dim3(a.B), dim3(SplitCfg<H>::NT), 0, st, a, al,
                       per);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
template <bool CLOSED, bool INLIN = false>
static int launch_split_t(const KArgs& a, double* sws, hipStream_t st) {
    const int n = 2 * a.c.N;
    double* al = align16(sws);
    const size_t per = split_ws_doubles(a.c.N);
    if (split_h(n) == 40) return launch_one<40, CLOSED, INLIN>(a, al, per, st);
    if (split_h(n) == 48) return launch_one<48, CLOSED, INLIN>(a, al, per, st);
    return launch_one<64, CLOSED, INLIN>(a, al, per, st);
}

// The fused closed loop (a.nsteps steps; the queue, order and lead set up by the caller): one workgroup per resident
// slot (occupancy x CUs; at least ceil(B / TRAJ_FUSED_MAX_PER_WG), at most B), each with its own P scratch.  Per device
// the slot count is asked of the occupancy API once.
template <int H>
static int launch_fused_h(const KArgs& a, double* al, size_t per, hipStream_t st) {
    static int slots_per_cu[64] = {0};
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return -3;
    if (!slots_per_cu[dev]) {
        int nb = 0, ncu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, solve_split_kernel<H, true, true>, SplitCfg<H>::NT, 0) !=
                hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -3;
        slots_per_cu[dev] = nb < 1 ? 1 : nb;
        cus[dev] = ncu < 1 ? 1 : ncu;
    }
    int G = a.fused_grid > 0 ? a.fused_grid : slots_per_cu[dev] * cus[dev];
    if (G > a.B) G = a.B;
    const int minG = (a.B + TRAJ_FUSED_MAX_PER_WG - 1) / TRAJ_FUSED_MAX_PER_WG;
    if (G < minG) G = minG;
    if (a.dbg)   // the stamped instance (tools/split_phase.py)
        hipLaunchKernelGGL((solve_split_kernel<H, true, true, true, true>), dim3(G), dim3(SplitCfg<H>::NT), 0, st, a,
                           al, per);
    else
        hipLaunchKernelGGL((solve_split_kernel<H, true, true>), dim3(G), dim3(SplitCfg<H>::NT), 0, st, a, al, per);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_split_step(const KArgs& a, double* sws, hipStream_t st, bool inlin) {
    return inlin ? launch_split_t<false, true>(a, sws, st) : launch_split_t<false>(a, sws, st);
}
int launch_split_closed(const KArgs& a, double* sws, hipStream_t st) { return launch_split_t<true>(a, sws, st); }
int launch_split_fused(const KArgs& a, double* sws, hipStream_t st) {
    const int n = 2 * a.c.N;
    double* al = align16(sws);
    const size_t per = split_ws_doubles(a.c.N);
    if (split_h(n) == 40) return launch_fused_h<40>(a, al, per, st);
    if (split_h(n) == 48) return launch_fused_h<48>(a, al, per, st);
    return launch_fused_h<64>(a, al, per, st);
}

}  // namespace tgmpc
