// trajmpc.hip -- C ABI of libtrajmpc.so (declared in include/trajmpc.h).
//
// Batched physics kernels (one thread per point) and the dispatch of the fused MPC kernel
// (mpc_kernel.h) by horizon capacity.  Built for gfx950 only:
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -shared -fPIC
#include <hip/hip_runtime.h>

#include <cmath>
#include <atomic>
#include <cstring>
#include <vector>

#include "../../include/trajmpc.h"
#include "mpc_common.h"
#include "mpc_general.h"
#include "mpc_long.h"
#include "mpc_split.h"   // (split_ws_doubles; the kernels are instantiated in split_inst.hip)
#include "mpc_linearize.h"
#include "physics.h"

namespace tgmpc {

// ---------------------------------------------------------------- physics kernels

__global__ void tire_forces_kernel(traj_vehicle_params p, int B, const double* x, const double* u, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double Fyf, Fyr, Frx;
    tire_forces(p, x[6 * i + 3], x[6 * i + 4], x[6 * i + 5], u[2 * i], u[2 * i + 1], Fyf, Fyr, Frx);
    out[3 * i] = Fyf;
    out[3 * i + 1] = Fyr;
    out[3 * i + 2] = Frx;
}

__global__ void f_cont_kernel(traj_vehicle_params p, int B, const double* x, const double* u, double* xd) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double xs[6], us[2], f[6];
    for (int j = 0; j < 6; ++j) xs[j] = x[6 * i + j];
    us[0] = u[2 * i];
    us[1] = u[2 * i + 1];
    f_cont(p, xs, us, f);
    for (int j = 0; j < 6; ++j) xd[6 * i + j] = f[j];
}

// mpc_6stati.py:73-97 (all 16 central differences + f, like the reference)
__device__ void numjac(const traj_vehicle_params& p, const double* x, const double* u, double ex, double eu,
                       double* Jx, double* Ju, double* f) {
    double xp[6], xm[6], up[2], um[2], fp[6], fm[6];
    for (int i = 0; i < 6; ++i) {
        for (int j = 0; j < 6; ++j) {
            double dx = (j == i) ? ex : 0.0;
            xp[j] = x[j] + dx;
            xm[j] = x[j] - dx;
        }
        f_cont(p, xp, u, fp);
        f_cont(p, xm, u, fm);
        for (int r = 0; r < 6; ++r) Jx[r * 6 + i] = (fp[r] - fm[r]) / (2.0 * ex);
    }
    for (int i = 0; i < 2; ++i) {
        for (int j = 0; j < 2; ++j) {
            double du = (j == i) ? eu : 0.0;
            up[j] = u[j] + du;
            um[j] = u[j] - du;
        }
        f_cont(p, x, up, fp);
        f_cont(p, x, um, fm);
        for (int r = 0; r < 6; ++r) Ju[r * 2 + i] = (fp[r] - fm[r]) / (2.0 * eu);
    }
    f_cont(p, x, u, f);
}

__global__ void numjac_kernel(traj_vehicle_params p, int B, const double* x, const double* u, double ex, double eu,
                              double* Jx, double* Ju, double* f) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double xs[6], us[2], jx[36], ju[12], fv[6];
    for (int j = 0; j < 6; ++j) xs[j] = x[6 * i + j];
    us[0] = u[2 * i];
    us[1] = u[2 * i + 1];
    numjac(p, xs, us, ex, eu, jx, ju, fv);
    for (int j = 0; j < 36; ++j) Jx[36 * i + j] = jx[j];
    for (int j = 0; j < 12; ++j) Ju[12 * i + j] = ju[j];
    for (int j = 0; j < 6; ++j) f[6 * i + j] = fv[j];
}

// mpc_6stati.py:99-109
__global__ void lindisc_kernel(traj_vehicle_params p, int B, double Ts, const double* x, const double* u, double* Ad,
                               double* Bd, double* g) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    double xs[6], us[2], jx[36], ju[12], fv[6], A[36], Bm[12];
    for (int j = 0; j < 6; ++j) xs[j] = x[6 * i + j];
    us[0] = u[2 * i];
    us[1] = u[2 * i + 1];
    numjac(p, xs, us, 1e-5, 1e-5, jx, ju, fv);
    for (int r = 0; r < 6; ++r)
        for (int cc = 0; cc < 6; ++cc) A[r * 6 + cc] = ((r == cc) ? 1.0 : 0.0) + Ts * jx[r * 6 + cc];
    for (int j = 0; j < 12; ++j) Bm[j] = Ts * ju[j];
    for (int r = 0; r < 6; ++r) {
        double ax = 0.0, bu = 0.0;
        for (int cc = 0; cc < 6; ++cc) ax += A[r * 6 + cc] * xs[cc];
        for (int cc = 0; cc < 2; ++cc) bu += Bm[r * 2 + cc] * us[cc];
        g[6 * i + r] = xs[r] + Ts * fv[r] - ax - bu;
    }
    for (int j = 0; j < 36; ++j) Ad[36 * i + j] = A[j];
    for (int j = 0; j < 12; ++j) Bd[12 * i + j] = Bm[j];
}

__global__ void lateral_error_kernel(int B, const double* X, const double* Y, const double* Xr, const double* Yr,
                                     const double* Pr, double* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    out[i] = lateral_error(X[i], Y[i], Xr[i], Yr[i], Pr[i]);
}

// main.py:51-68 batched (one thread per trajectory: the x-advance is a running sum)
// (xs_stride: x_start[xs_stride b] -- 1 for traj_ref_window_batch, 6 for the closed loop's state rows)
__global__ void ref_window_kernel(PathArgs pa, int B, int N, double Ts, const double* x_start, int xs_stride,
                                  const double* vref, double* pref) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xs = x_start[(size_t)xs_stride * b];
    for (int k = 0; k <= N; ++k) {
        if (k > 0) xs = xs + vref[(size_t)(N + 1) * b + k - 1] * Ts;
        double y, dy;
        path_eval(pa, b, xs, y, dy);
        double* o = pref + ((size_t)(N + 1) * b + k) * 3;
        o[0] = xs;
        o[1] = y;
        o[2] = pm_atan(dy);
    }
}

// ---------------------------------------------------------------- closed-loop solve order
// Counting sort of the instances by a per-instance cost record (ADMM iterations: slot 2 = the last
// step's, slot 3 = the mean per step of the last fused launch; 25-iteration buckets, descending): a
// permutation whatever the workspace holds (non-finite keys land in bucket 0).
__global__ __launch_bounds__(1024) void order_kernel(const double* warm, int B, int* perm, int slot) {
    constexpr int NBK = 512;
    __shared__ int hist[NBK];
    __shared__ int offs[NBK];
    const int t = threadIdx.x;
    for (int i = t; i < NBK; i += 1024) hist[i] = 0;
    __syncthreads();
    auto key = [&](int i) -> int {
        const double v = fmin(fmax(warm[4 * (size_t)i + slot] / 25.0, 0.0), (double)(NBK - 1));
        return (int)v;
    };
    for (int i = t; i < B; i += 1024) atomicAdd(&hist[key(i)], 1);
    __syncthreads();
    if (t == 0) {
        int acc = 0;
        for (int k = NBK - 1; k >= 0; --k) {
            offs[k] = acc;
            acc += hist[k];
        }
    }
    __syncthreads();
    for (int i = t; i < B; i += 1024) perm[atomicAdd(&offs[key(i)], 1)] = i;
}

// ---------------------------------------------------------------- MPC dispatch

// per-capacity launchers (mpc_inst.hip compiled once per NN)
// Kernel capacities (QP variables, n = 2N): 16 / 32 / 40 one wave per instance, 80 two waves.  20 < N <= 40 runs
// capacity 80: a one-wave capacity-64 instance has no spare lanes for the receiver sweep and, at 64 doubles of K^-1
// per lane beside the chunked reads, spilled 780-830 B/lane at 512 registers; measured at B = 1024
// (profiles/r05_tiers.json) it ran N = 24 / 30 / 32 at 0.43 / 0.34 / 0.35 M steps/s against 0.56 / 0.47 / 0.46 M on
// capacity 80, so it is not built (TGMPC_CAP64=1 brings it back for experiments)
#ifndef TGMPC_CAP64
#define TGMPC_CAP64 0
#endif
#if TGMPC_CAP64
#define TGMPC_CAPACITIES(X) X(16) X(32) X(40) X(64) X(80)
#else
#define TGMPC_CAPACITIES(X) X(16) X(32) X(40) X(80)
#endif
#define TGMPC_DECL(NNV) int launch_mpc_##NNV(const KArgs& a, hipStream_t st, int mode);
TGMPC_CAPACITIES(TGMPC_DECL)
#undef TGMPC_DECL

// rollout (one thread per instance) + central-difference linearization (one thread per stage)
static void launch_linearize(const KArgs& a, hipStream_t st, bool closed) {
    const int nr = (a.B + 63) / 64, nj = (a.B * a.c.N + 63) / 64;
    if (closed) {
        hipLaunchKernelGGL(rollout_kernel<true>, dim3(nr), dim3(64), 0, st, a);
        hipLaunchKernelGGL(jac_kernel<true>, dim3(nj), dim3(256), 0, st, a);
    } else {
        hipLaunchKernelGGL(rollout_kernel<false>, dim3(nr), dim3(64), 0, st, a);
        hipLaunchKernelGGL(jac_kernel<false>, dim3(nj), dim3(256), 0, st, a);
    }
}

// workspace layout: A [B,N,36] | B [B,N,12] | g [B,N,6] | rollout record [B,N,12] | warm [B,4] | order int[B]
static void carve_workspace(KArgs& a, void* ws, int B, int N) {
    a.wsA = (double*)ws;
    a.wsB = a.wsA + (size_t)B * N * 36;
    a.wsg = a.wsB + (size_t)B * N * 12;
    a.wsXF = a.wsg + (size_t)B * N * 6;
    a.wsWarm = a.wsXF + (size_t)B * N * 12;
    a.Ad = a.wsA; a.Bd = a.wsB; a.gd = a.wsg;
}

static int launch_mpc(const KArgs& a, hipStream_t st, int mode) {
    const int n = 2 * a.c.N;
#define TGMPC_CASE(NNV) \
    if (n <= NNV) return launch_mpc_##NNV(a, st, mode);
    TGMPC_CAPACITIES(TGMPC_CASE)
#undef TGMPC_CASE
    return TRAJ_E_ARG;
}

// state bounds (mpc_6stati.py:208-213) with at least one finite side
static bool state_bounds_active(const traj_mpc_config* c) {
    for (int i = 0; i < 6; ++i) {
        if (c->has_x_lo && c->x_lo[i] > -INFTY) return true;
        if (c->has_x_hi && c->x_hi[i] < INFTY) return true;
    }
    return false;
}

// allow_sb: the caller can run the general solver (state bounds, horizons past TRAJ_MAX_N); the closed-loop
// entry points cannot
static int check_cfg(const traj_mpc_config* c, bool allow_sb = false) {
    if (!c) return TRAJ_E_ARG;
    if (c->N < 1 || c->N > TRAJ_MAX_N_GENERAL) return TRAJ_E_ARG;
    if (c->N > TRAJ_MAX_N && !allow_sb) return TRAJ_E_UNSUPPORTED;
    if (!(c->Ts > 0.0) || c->max_iter < 1 || c->check_interval < 1 || c->scaling_iters < 0) return TRAJ_E_ARG;
    if (c->polish_mode != 0 && c->polish_mode != 1) return TRAJ_E_ARG;
    if (!allow_sb && state_bounds_active(c)) return TRAJ_E_UNSUPPORTED;
    return TRAJ_OK;
}

// the general solver (mpc_general.h) for configurations with state bounds: its per-instance scratch is
// the caller's (traj_mpc_sb_workspace_bytes), like every other buffer -- no allocation per call
static int launch_general(const KArgs& a, double* gws, hipStream_t st) {
    const size_t per = gen_ws_doubles(a.c.N);
    if (2 * a.c.N <= 64 * GEN_RMAX_SMALL)
        hipLaunchKernelGGL(solve_gen_kernel<GEN_RMAX_SMALL>, dim3(a.B), dim3(GEN_NT), 0, st, a, gws, per);
    else
        hipLaunchKernelGGL(solve_gen_kernel<GEN_RMAX>, dim3(a.B), dim3(GEN_NT), 0, st, a, gws, per);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

// the long-horizon kernel (mpc_long.h): TRAJ_MAX_N < N <= TRAJ_MAX_N_LONG without state bounds; its per-instance
// scratch (the scaled P, and K^-1 past LONG_NKL) is the caller's, in the same region as the general solver's.
// CLOSED: one closed-loop step (window from the state, warm rho, plant update) -- traj_closed_loop_step / _run.
template <bool CLOSED>
static int launch_long(const KArgs& a, double* lws, hipStream_t st) {
    const int N = a.c.N;
    const size_t per = long_ws_doubles(N);
    if (2 * N <= LONG_NKL) {
        const size_t lds = long_lds_bytes(N);
        // the dynamic-LDS attribute is set once per device (it belongs to the function's per-device code object); the
        // flags are atomics, so concurrent callers on several host threads at worst set it twice
        static std::atomic<bool> attr[64];
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return TRAJ_E_LAUNCH;
        if (dev < 0 || dev >= 64 || !attr[dev].load(std::memory_order_acquire)) {
            if (hipFuncSetAttribute(reinterpret_cast<const void*>(&solve_long_kernel<true, CLOSED>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(LONG_NKL * LONG_NKL * sizeof(double))) != hipSuccess)
                return TRAJ_E_LAUNCH;
            if (dev >= 0 && dev < 64) attr[dev].store(true, std::memory_order_release);
        }
        hipLaunchKernelGGL((solve_long_kernel<true, CLOSED>), dim3(a.B), dim3(LONG_NT), lds, st, a, lws, per);
    } else if (2 * N <= LONG_NT) {
        hipLaunchKernelGGL((solve_long_kernel<false, CLOSED>), dim3(a.B), dim3(LONG_NT), 0, st, a, lws, per);
    } else {   // 128 < N <= TRAJ_MAX_N_LONG: the 512-thread instance (round 6)
        hipLaunchKernelGGL((solve_long_kernel<false, CLOSED, LONG_NT2>), dim3(a.B), dim3(LONG_NT2), 0, st, a, lws, per);
    }
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

// the row-split kernel (mpc_split.h; split_inst.hip, its own translation unit built without machine LICM like the
// other register-resident solvers): TRAJ_MAX_N < N <= TRAJ_MAX_N_SPLIT without state bounds
int launch_split_step(const KArgs& a, double* sws, hipStream_t st, bool inlin);
int launch_split_closed(const KArgs& a, double* sws, hipStream_t st);
int launch_split_fused(const KArgs& a, double* sws, hipStream_t st);
template <bool CLOSED>
static int launch_split(const KArgs& a, double* sws, hipStream_t st) {
    return CLOSED ? launch_split_closed(a, sws, st) : launch_split_step(a, sws, st, false);
}

// fused run queue order: the heaviest 10 % of the instances (by the previous launch's mean ADMM
// iterations) one step ahead of the level front (mpc_solve.h; measured +1.9 % at the driver's 20-step
// command, neutral at 200 steps)
#ifndef TGMPC_LEAD_STEPS
#define TGMPC_LEAD_STEPS 1
#endif
#ifndef TGMPC_LEAD_PERMILLE
#define TGMPC_LEAD_PERMILLE 100
#endif
static long long* g_dbg = nullptr;  // diagnostics buffer (traj_debug_set_stamps)
static long long* g_dbg_items = nullptr;  // fused-run item timeline (traj_debug_set_item_stamps)
static int g_fused_grid = 0;        // traj_debug_fused_grid
// fused runs of at least this many steps use the 3-waves-per-SIMD kernel (capacity 40; 0 = never).  Round 3 measured
// it ahead over long launches (200 steps: 14.35 M vs 13.51 M steps/s; behind at 20 and 100 steps, where a launch is
// bound by its heaviest instances' chains); since round 4's arithmetic work the 2-wave instance matches it there
// (round 5, 240 steps: 16.26-16.28 M vs 16.32-16.39 M) without its 156 B/lane of scratch, so it runs every launch
// length and the 3-wave instance is opt-in (traj_debug_fused_waves(3)) -- DESIGN.md section 5
#ifndef TRAJ_FUSED_W3_MIN_STEPS
#define TRAJ_FUSED_W3_MIN_STEPS 0
#endif
static int g_fused_waves = 0;       // traj_debug_fused_waves: 0 = by launch length, 2 or 3 = forced
static int g_spin_limit = 1 << 22;  // traj_debug_spin_limit: polls before a fused hand-off is declared lost
static int g_lead_steps = TGMPC_LEAD_STEPS, g_lead_permille = TGMPC_LEAD_PERMILLE;   // traj_debug_queue_lead
// fused run: a workgroup that completes an instance's step takes the instance's next step itself while that step is
// at most this many levels past the queue's draw front (mpc_solve.h); 0 = every item from the queue in its order.
// Off by default: at N = 20 it only adds contention (8 levels: 11.9 M vs 12.8 M); at config 3 it moves where the
// launch's iteration-cap chains fall -- +6.6 % on the bench's workload at 8 levels, -2.4 .. +2 % on three others
// (profiles/r05_run_ahead*.json)
#ifndef TGMPC_RUN_AHEAD
#define TGMPC_RUN_AHEAD 0
#endif
static int g_run_ahead = TGMPC_RUN_AHEAD;   // traj_debug_run_ahead
// horizons up to which TRAJ_MAX_N < N runs the row-split kernel (mpc_split.h) instead of the long-horizon one
// (traj_debug_split_max_n: 0 sends every N > TRAJ_MAX_N to the long-horizon kernel; the two agree to the step bars)
static int g_split_max_n = TRAJ_MAX_N_SPLIT;
// horizons from which the step and the closed loop (fused and per step) run the row-split kernel: default
// TRAJ_SPLIT_MIN_N = 21, so that 20 < N <= TRAJ_MAX_N_SPLIT all run it -- at config 3 (N = 40, mixed references) it is
// 1.09-1.10 M steps/s against the capacity-80 kernel's 1.02 M (its iteration-cap chains at 0.76 instead of 1.16 us per
// ADMM iteration), within +-3 % of it on spline references at N = 24 / 32 / 40 (profiles/r06_split_probe*.json);
// traj_debug_split_min_n(TRAJ_MAX_N + 1) sends 20 < N <= TRAJ_MAX_N back to the capacity-80 kernel
static int g_split_min_n = TRAJ_SPLIT_MIN_N;
static bool split_route(const traj_mpc_config* c) {
    return !state_bounds_active(c) && c->N >= g_split_min_n && c->N <= g_split_max_n;
}
// the row-split kernel's P scratch inside the workspace (after the base part): every horizon it can run, whatever the
// routing, so that traj_mpc_workspace_bytes does not depend on a debug switch
static size_t split_bytes(int B, int N) {
    return (N >= 21 && N <= TRAJ_MAX_N_SPLIT) ? ((size_t)B * split_ws_doubles(N) + 2) * sizeof(double) : 0;
}
// traj_debug_step_linearize: the step's linearization inside the solve launch.  An atomic: a test that flips it may run
// beside other callers of the library; each traj_mpc_step_batch reads it once.
static std::atomic<int> g_step_inlin{1};

// per-kernel timing of traj_closed_loop_step (traj_debug_kernel_timing): 5 events per step bracket
// rollout | jac | order | solve on the launch stream
static std::vector<hipEvent_t> g_ev;
static int g_ev_used = 0;
static inline void stamp(int k, hipStream_t st) {
    if ((size_t)(5 * g_ev_used + k) < g_ev.size()) (void)hipEventRecord(g_ev[5 * g_ev_used + k], st);
}

static inline unsigned nblk(int B, int bs) { return (unsigned)((B + bs - 1) / bs); }

}  // namespace tgmpc

using namespace tgmpc;

extern "C" {

int traj_abi_version(void) { return TRAJMPC_ABI_VERSION; }

int traj_debug_set_stamps(long long* buf) {
    g_dbg = buf;
    return TRAJ_OK;
}

int traj_debug_set_item_stamps(long long* buf) {
    g_dbg_items = buf;
    return TRAJ_OK;
}

int traj_debug_fused_grid(int workgroups) {
    if (workgroups < 0) return TRAJ_E_ARG;
    g_fused_grid = workgroups;
    return TRAJ_OK;
}

int traj_debug_fused_waves(int waves) {
    if (waves < 0 || waves > 3) return TRAJ_E_ARG;
    g_fused_waves = waves;
    return TRAJ_OK;
}

int traj_debug_queue_lead(int steps, int per_mille) {
    if (steps < 0 || per_mille < 0 || per_mille > 1000) return TRAJ_E_ARG;
    g_lead_steps = steps;
    g_lead_permille = per_mille;
    return TRAJ_OK;
}

int traj_debug_run_ahead(int levels) {
    if (levels < 0) return TRAJ_E_ARG;
    g_run_ahead = levels;
    return TRAJ_OK;
}

int traj_debug_split_min_n(int n_min) {
    if (n_min < 21 || n_min > TRAJ_MAX_N + 1) return TRAJ_E_ARG;
    g_split_min_n = n_min;
    return TRAJ_OK;
}

int traj_debug_split_max_n(int n_max) {
    if (n_max < 0 || n_max > TRAJ_MAX_N_SPLIT) return TRAJ_E_ARG;
    g_split_max_n = n_max;
    return TRAJ_OK;
}

int traj_debug_step_linearize(int in_kernel) {
    if (in_kernel != 0 && in_kernel != 1) return TRAJ_E_ARG;
    g_step_inlin.store(in_kernel, std::memory_order_relaxed);
    return TRAJ_OK;
}

int traj_debug_spin_limit(int polls) {
    if (polls < 0) return TRAJ_E_ARG;
    g_spin_limit = polls ? polls : (1 << 22);
    return TRAJ_OK;
}

int traj_debug_kernel_timing(int max_steps) {
    for (hipEvent_t e : g_ev) (void)hipEventDestroy(e);
    g_ev.clear();
    g_ev_used = 0;
    if (max_steps < 0) return TRAJ_E_ARG;
    g_ev.resize((size_t)5 * max_steps);
    for (auto& e : g_ev)
        if (hipEventCreate(&e) != hipSuccess) return TRAJ_E_LAUNCH;
    return TRAJ_OK;
}

int traj_debug_kernel_times(double* ms, int* n_steps) {
    if (!ms || !n_steps) return TRAJ_E_ARG;
    for (int k = 0; k < 4; ++k) ms[k] = 0.0;
    *n_steps = g_ev_used;
    for (int s = 0; s < g_ev_used; ++s) {
        hipEvent_t* e = &g_ev[5 * (size_t)s];
        if (hipEventSynchronize(e[4]) != hipSuccess) return TRAJ_E_LAUNCH;
        for (int k = 0; k < 4; ++k) {
            float t = 0.f;
            if (hipEventElapsedTime(&t, e[k], e[k + 1]) != hipSuccess) return TRAJ_E_LAUNCH;
            ms[k] += t;
        }
    }
    if (g_ev_used > 0)
        for (int k = 0; k < 4; ++k) ms[k] /= g_ev_used;
    g_ev_used = 0;
    return TRAJ_OK;
}

const char* traj_status_string(int s) {
    switch (s) {
        case TRAJ_STATUS_OPTIMAL: return "optimal";
        case TRAJ_STATUS_OPTIMAL_INACCURATE: return "optimal_inaccurate";
        case TRAJ_STATUS_USER_LIMIT: return "user_limit";
        case TRAJ_STATUS_INFEASIBLE: return "infeasible";
        case TRAJ_STATUS_INFEASIBLE_INACCURATE: return "infeasible_inaccurate";
        case TRAJ_STATUS_UNBOUNDED: return "unbounded";
        case TRAJ_STATUS_SOLVER_ERROR: return "Solver Error: SolverError";
        default: return "unknown";
    }
}

const char* traj_error_string(int e) {
    switch (e) {
        case TRAJ_OK: return "ok";
        case TRAJ_E_ARG: return "invalid argument";
        case TRAJ_E_UNSUPPORTED: return "unsupported configuration";
        case TRAJ_E_LAUNCH: return "HIP launch failure";
        case TRAJ_E_HANDOFF: return "fused closed loop: an instance hand-off timed out (results invalid)";
        default: return "unknown error";
    }
}

int traj_default_params(traj_vehicle_params* p) {
    if (!p) return TRAJ_E_ARG;
    p->Cm1 = 0.287; p->Cm2 = 0.0545; p->Cr0 = 0.0518; p->Cr2 = 0.00035;
    p->Br = 3.3852; p->Cr = 1.2691; p->Dr = 0.1737;
    p->Bf = 2.579; p->Cf = 1.2; p->Df = 0.192;
    p->m = 0.041; p->Iz = 27.8e-6; p->lf = 0.029; p->lr = 0.033;
    p->g = 9.81; p->maxAlpha = 0.6; p->vx_zero = 0.3;
    return TRAJ_OK;
}

int traj_default_config(traj_mpc_config* c, int N, double Ts) {
    if (!c) return TRAJ_E_ARG;
    std::memset(c, 0, sizeof(*c));
    c->N = N; c->Ts = Ts;
    c->q_c = 6.0; c->q_phi = 0.5; c->q_vx = 0.5;
    c->R[0] = 0.02; c->R[3] = 2.0;
    c->Rd[0] = 0.01; c->Rd[3] = 5.0;
    c->u_lo[0] = -1.0; c->u_hi[0] = 1.0; c->u_lo[1] = -0.6; c->u_hi[1] = 0.6;
    c->du_lo[0] = -0.5; c->du_hi[0] = 0.5; c->du_lo[1] = -0.3; c->du_hi[1] = 0.3;
    c->eps_abs = 1e-5; c->eps_rel = 1e-5; c->eps_prim_inf = 1e-4;
    c->rho = 0.1; c->sigma = 1e-6; c->alpha = 1.6; c->delta = 1e-6;
    c->max_iter = 10000; c->check_interval = 25; c->scaling_iters = 10;
    c->polish = 1; c->polish_refine_iter = 3; c->adaptive_rho = 1; c->adaptive_rho_tol = 5.0;
    c->polish_mode = 0; c->polish_max_pass = 8; c->cert_tol = 1e-9; c->polish_max_rounds = 2;
    c->warm_start = 1;
    return TRAJ_OK;
}

int traj_tire_forces_batch(const traj_vehicle_params* p, int B, const double* x, const double* u, double* out,
                           void* stream) {
    if (!p || B < 0 || (B > 0 && (!x || !u || !out))) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    hipLaunchKernelGGL(tire_forces_kernel, dim3(nblk(B, 256)), dim3(256), 0, (hipStream_t)stream, *p, B, x, u, out);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_f_cont_batch(const traj_vehicle_params* p, int B, const double* x, const double* u, double* xdot,
                      void* stream) {
    if (!p || B < 0 || (B > 0 && (!x || !u || !xdot))) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    hipLaunchKernelGGL(f_cont_kernel, dim3(nblk(B, 256)), dim3(256), 0, (hipStream_t)stream, *p, B, x, u, xdot);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_numerical_jacobian_batch(const traj_vehicle_params* p, int B, const double* x, const double* u,
                                  double eps_x, double eps_u, double* Jx, double* Ju, double* f, void* stream) {
    if (!p || B < 0 || (B > 0 && (!x || !u || !Jx || !Ju || !f))) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    hipLaunchKernelGGL(numjac_kernel, dim3(nblk(B, 128)), dim3(128), 0, (hipStream_t)stream, *p, B, x, u, eps_x,
                       eps_u, Jx, Ju, f);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_linearize_discretize_batch(const traj_vehicle_params* p, int B, double Ts, const double* xbar,
                                    const double* ubar, double* Ad, double* Bd, double* g, void* stream) {
    if (!p || B < 0 || (B > 0 && (!xbar || !ubar || !Ad || !Bd || !g))) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    hipLaunchKernelGGL(lindisc_kernel, dim3(nblk(B, 128)), dim3(128), 0, (hipStream_t)stream, *p, B, Ts, xbar, ubar,
                       Ad, Bd, g);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

int traj_lateral_error_batch(int B, const double* X, const double* Y, const double* Xref, const double* Yref,
                             const double* phiref, double* out, void* stream) {
    if (B < 0 || (B > 0 && (!X || !Y || !Xref || !Yref || !phiref || !out))) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    hipLaunchKernelGGL(lateral_error_kernel, dim3(nblk(B, 256)), dim3(256), 0, (hipStream_t)stream, B, X, Y, Xref,
                       Yref, phiref, out);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

static size_t ws_base_bytes(int B, int N);

// lin: the step (linearization in the library, `ws` holds its hand-off + the state-bound scratch after
// it); !lin: the QP half (Ad / Bd / g given, `ws` is only the state-bound scratch, may be NULL without
// state bounds)
static int mpc_common(const traj_vehicle_params* p, const traj_mpc_config* c, int B, const double* x0,
                      const double* u_prev, const double* path_ref, const double* vref, const double* Ad,
                      const double* Bd, const double* g, double* u_cmd, int* status, double* objective,
                      double* X_opt, double* U_opt, int* iters, int* polished, void* ws, size_t ws_bytes,
                      void* stream, bool lin) {
    if (!p || B < 0) return TRAJ_E_ARG;
    int e = check_cfg(c, true);
    if (e) return e;
    if (B == 0) return TRAJ_OK;
    if (!x0 || !u_prev || !path_ref || !vref || !u_cmd || !status) return TRAJ_E_ARG;
    if (!lin && (!Ad || !Bd || !g)) return TRAJ_E_ARG;
    // which solver (include/trajmpc.h tiers): the general one (state bounds, or N > TRAJ_MAX_N_LONG), the long-horizon
    // one (TRAJ_MAX_N_SPLIT < N <= TRAJ_MAX_N_LONG), the row-split one (split_route; the QP entry point up to TRAJ_MAX_N
    // keeps the capacity-80 kernel, which needs no scratch), or the register-resident ones.  Scratch: the step's
    // workspace holds the row-split kernel's (traj_mpc_workspace_bytes); the others' follows it (+ sb bytes), as does
    // the QP entry point's whole scratch
    const bool use_split = split_route(c) && (lin || c->N > TRAJ_MAX_N);
    const bool gen_long = state_bounds_active(c) || (c->N > TRAJ_MAX_N && !use_split);
    const bool sb = gen_long || use_split;
    const size_t base = lin ? ws_base_bytes(B, c->N) : 0;
    const size_t need = lin ? base + (gen_long ? traj_mpc_sb_workspace_bytes(B, c->N)
                                               : (use_split ? split_bytes(B, c->N) : 0))
                            : (sb ? traj_mpc_sb_workspace_bytes(B, c->N) : 0);
    if (need > 0 && (!ws || ws_bytes < need)) return TRAJ_E_ARG;
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.p = *p;
    a.c = *c;
    a.B = B;
    a.x0 = x0; a.u_prev = u_prev; a.path_ref = path_ref; a.vref = vref;
    if (lin) {
        carve_workspace(a, ws, B, c->N);
        a.wsWarm = nullptr;
    } else {
        a.Ad = Ad; a.Bd = Bd; a.gd = g;
    }
    a.u_cmd = u_cmd; a.status = status; a.objective = objective; a.X_opt = X_opt; a.U_opt = U_opt;
    a.iters = iters; a.polished = polished;
    a.dbg = g_dbg;
    // the step: one launch with the linearization in the workgroup (mode 4), or rollout_kernel + jac_kernel +
    // the solve (traj_debug_step_linearize(0); the general solver always reads A/B/g from the workspace)
    // (the row-split kernel likewise when it runs the step; the QP entry point and the other scratch solvers read A/B/g
    // from the workspace)
    const int inlin = g_step_inlin.load(std::memory_order_relaxed);
    const bool split_inlin = use_split && lin && inlin;
    if (lin && ((sb && !split_inlin) || !inlin)) launch_linearize(a, (hipStream_t)stream, false);
    if (sb) {
        double* const sws = (double*)((char*)ws + base);
        if (use_split) return launch_split_step(a, sws, (hipStream_t)stream, split_inlin) ? TRAJ_E_LAUNCH : TRAJ_OK;
        if (!state_bounds_active(c) && c->N <= TRAJ_MAX_N_LONG) return launch_long<false>(a, sws, (hipStream_t)stream);
        return launch_general(a, sws, (hipStream_t)stream);
    }
    return launch_mpc(a, (hipStream_t)stream, lin ? (inlin ? 4 : 0) : 1);
}

// A/B/g hand-off (54 N doubles), rollout record (12 N), warm-start record (4), closed-loop order
// (1 int), fused-run step queue (counter, error flag, completed and claimed steps per instance); a multiple of 8
static size_t ws_base_bytes(int B, int N) {
    return ((size_t)B * (size_t)N * 66 + (size_t)B * 4) * sizeof(double) +
           ((((size_t)B * 3 + 2) * sizeof(int) + 7) & ~(size_t)7);
}

size_t traj_mpc_workspace_bytes(int B, int N) {
    if (B < 0 || N < 0) return 0;
    return ws_base_bytes(B, N) + split_bytes(B, N);
}

size_t traj_mpc_sb_workspace_bytes(int B, int N) {
    if (B < 0 || N < 1 || N > TRAJ_MAX_N_GENERAL) return 0;
    return (size_t)B * gen_ws_doubles(N) * sizeof(double);
}

int traj_mpc_step_batch(const traj_vehicle_params* p, const traj_mpc_config* c, int B, const double* x0,
                        const double* u_prev, const double* path_ref, const double* vref, double* u_cmd,
                        int* status, double* objective, double* X_opt, double* U_opt, int* iters, int* polished,
                        void* workspace, size_t workspace_bytes, void* stream) {
    return mpc_common(p, c, B, x0, u_prev, path_ref, vref, nullptr, nullptr, nullptr, u_cmd, status, objective,
                      X_opt, U_opt, iters, polished, workspace, workspace_bytes, stream, true);
}

int traj_mpc_qp_batch(const traj_vehicle_params* p, const traj_mpc_config* c, int B, const double* x0,
                      const double* u_prev, const double* path_ref, const double* vref, const double* Ad,
                      const double* Bd, const double* g, double* u_cmd, int* status, double* objective,
                      double* X_opt, double* U_opt, int* iters, int* polished, void* workspace,
                      size_t workspace_bytes, void* stream) {
    return mpc_common(p, c, B, x0, u_prev, path_ref, vref, Ad, Bd, g, u_cmd, status, objective, X_opt, U_opt, iters,
                      polished, workspace, workspace_bytes, stream, false);
}

static bool paths_ok(const traj_paths* ps) {
    return ps && ps->kind && ps->pc && (ps->kmax < 2 || (ps->nk && ps->xk && ps->coef));
}

int traj_ref_window_batch(const traj_paths* paths, int B, int N, double Ts, const double* x_start,
                          const double* vref, double* path_ref, void* stream) {
    if (B < 0 || N < 1 || !paths_ok(paths)) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!x_start || !vref || !path_ref) return TRAJ_E_ARG;
    PathArgs pa{paths->kmax, paths->kind, paths->pc, paths->nk, paths->xk, paths->coef};
    hipLaunchKernelGGL(ref_window_kernel, dim3(nblk(B, 128)), dim3(128), 0, (hipStream_t)stream, pa, B, N, Ts,
                       x_start, 1, vref, path_ref);
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

// The closed loop's horizons: N <= TRAJ_MAX_N on the register-resident kernels (fused or per step), TRAJ_MAX_N < N <=
// TRAJ_MAX_N_LONG on the long-horizon kernel, one step per launch sequence (rollout_kernel + jac_kernel + the closed
// solve_long_kernel).  The long tier needs the step's scratch beside the workspace, as the step entry point does:
// traj_mpc_workspace_bytes + traj_mpc_sb_workspace_bytes.  With state bounds (mpc_6stati.py:208-213; main.py passes
// none), or past TRAJ_MAX_N_LONG up to TRAJ_MAX_N_GENERAL, one step per launch sequence on the general solver
// (closed_step_sb below).
// (past TRAJ_MAX_N_LONG, or with state bounds: the general solver, closed_step_sb)
static bool closed_general(const traj_mpc_config* c) { return state_bounds_active(c) || c->N > TRAJ_MAX_N_LONG; }
static int check_cfg_closed(const traj_mpc_config* c) {
    if (c && (c->N > TRAJ_MAX_N || split_route(c) || state_bounds_active(c))) return check_cfg(c, true);
    return check_cfg(c);
}
// state bounds: the general solver's scratch after the workspace's base part (as the step's), then the step's window
// [B, N+1, 3], u_cmd [B, 2] and a status row [B] (int)
static size_t closed_sb_extra_off(int B, int N) { return ws_base_bytes(B, N) + traj_mpc_sb_workspace_bytes(B, N); }
static size_t closed_sb_bytes(int B, int N) {
    const size_t e = closed_sb_extra_off(B, N) + ((size_t)B * (3 * (size_t)(N + 1) + 2) + ((size_t)B + 1) / 2) * sizeof(double);
    const size_t w = traj_mpc_workspace_bytes(B, N);
    return e > w ? e : w;
}
static size_t closed_ws_bytes(const traj_mpc_config* c, int B) {
    const int N = c->N;   // (the row-split kernel's scratch is in traj_mpc_workspace_bytes; the long-horizon one's follows)
    if (closed_general(c)) return closed_sb_bytes(B, N);
    return traj_mpc_workspace_bytes(B, N) + ((N > TRAJ_MAX_N && !split_route(c)) ? traj_mpc_sb_workspace_bytes(B, N) : 0);
}
// one long-horizon closed-loop step on a's state (a.t = the step, a.status / a.iters = this step's [B] rows)
static int closed_step_long(const KArgs& a, void* ws, hipStream_t st) {
    stamp(0, st);
    launch_linearize(a, st, true);
    stamp(1, st);
    stamp(2, st);
    stamp(3, st);
    double* const sws = (double*)((char*)ws + ws_base_bytes(a.B, a.c.N));
    const int e = split_route(&a.c) ? launch_split<true>(a, sws, st) : launch_long<true>(a, sws, st);
    stamp(4, st);
    if ((size_t)(5 * g_ev_used + 4) < g_ev.size()) ++g_ev_used;
    return e;
}

// One closed-loop step on the general solver (state bounds, or N > TRAJ_MAX_N_LONG): the step entry point's launches on the loop's own state -- the window
// (ref_window_kernel on x[:, 0]), the linearization and the general solver (whose u_cmd carries mpc_step's u_prev
// fallback, mpc_6stati.py:257-262) -- then the plant update and the history (closed_sb_plant_kernel: the closed kernels'
// tail, main.py:97-101).  Each step is a fresh mpc_step call, as the reference's loop makes it: cold rho, no warm-start
// record (warm_start has nothing to carry here); the applied u is the step entry point's on the same state, bit for bit.
__global__ void closed_sb_plant_kernel(const KArgs a, const double* u_cmd) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.B) return;
    double xs[6], f[6], u[2] = {u_cmd[2 * (size_t)b], u_cmd[2 * (size_t)b + 1]};
    for (int i = 0; i < 6; ++i) xs[i] = a.x_state[6 * (size_t)b + i];
    f_cont(a.p, xs, u, f);
    for (int i = 0; i < 6; ++i) {
        const double xn = xs[i] + a.c.Ts * f[i];
        a.x_state[6 * (size_t)b + i] = xn;
        if (a.hist_x) a.hist_x[((size_t)b * (a.hist_T + 1) + a.t + 1) * 6 + i] = xn;
    }
    a.u_state[2 * (size_t)b] = u[0];
    a.u_state[2 * (size_t)b + 1] = u[1];
    if (a.hist_u) {
        a.hist_u[((size_t)b * a.hist_T + a.t) * 2] = u[0];
        a.hist_u[((size_t)b * a.hist_T + a.t) * 2 + 1] = u[1];
    }
}
static int closed_step_sb(const KArgs& a0, void* ws, hipStream_t st) {
    const int B = a0.B, N = a0.c.N;
    double* const sws = (double*)((char*)ws + ws_base_bytes(B, N));
    double* const pr = (double*)((char*)ws + closed_sb_extra_off(B, N));
    double* const uc = pr + (size_t)B * 3 * (N + 1);
    int* const sbuf = (int*)(uc + (size_t)B * 2);
    stamp(0, st);
    hipLaunchKernelGGL(ref_window_kernel, dim3(nblk(B, 128)), dim3(128), 0, st, a0.path, B, N, a0.c.Ts,
                       (const double*)a0.x_state, 6, a0.vref, pr);
    KArgs a = a0;
    a.x0 = a0.x_state;
    a.u_prev = a0.u_state;
    a.path_ref = pr;
    a.u_cmd = uc;
    a.status = a0.status ? a0.status : sbuf;
    a.objective = nullptr; a.X_opt = nullptr; a.U_opt = nullptr; a.polished = nullptr;
    a.wsWarm = nullptr;
    a.perm = nullptr;
    launch_linearize(a, st, false);
    stamp(1, st);
    stamp(2, st);
    stamp(3, st);
    int e = launch_general(a, sws, st);
    if (e) return e;
    hipLaunchKernelGGL(closed_sb_plant_kernel, dim3(nblk(B, 64)), dim3(64), 0, st, a0, (const double*)uc);
    stamp(4, st);
    if ((size_t)(5 * g_ev_used + 4) < g_ev.size()) ++g_ev_used;
    return hipGetLastError() == hipSuccess ? TRAJ_OK : TRAJ_E_LAUNCH;
}

size_t traj_closed_loop_workspace_bytes(const traj_mpc_config* c, int B) {
    if (!c || B < 0 || check_cfg_closed(c)) return 0;
    return closed_ws_bytes(c, B);
}

int traj_closed_loop_step(const traj_vehicle_params* p, const traj_mpc_config* c, const traj_paths* paths, int B,
                          double* x, double* u_prev, const double* vref, int t, int hist_T, double* hist_x,
                          double* hist_u, int* status, int* iters, void* workspace, size_t workspace_bytes,
                          void* stream) {
    if (!p || B < 0 || !paths_ok(paths)) return TRAJ_E_ARG;
    int e = check_cfg_closed(c);
    if (e) return e;
    if (B == 0) return TRAJ_OK;
    if (!x || !u_prev || !vref) return TRAJ_E_ARG;
    if (!workspace || workspace_bytes < closed_ws_bytes(c, B)) return TRAJ_E_ARG;
    if ((hist_x || hist_u) && (t < 0 || t >= hist_T)) return TRAJ_E_ARG;
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.p = *p;
    a.c = *c;
    a.B = B;
    a.vref = vref;
    a.path = PathArgs{paths->kmax, paths->kind, paths->pc, paths->nk, paths->xk, paths->coef};
    a.x_state = x;
    a.u_state = u_prev;
    a.t = t;
    a.hist_T = hist_T;
    a.hist_x = hist_x;
    a.hist_u = hist_u;
    a.status = status;
    a.iters = iters;
    a.dbg = g_dbg;
    carve_workspace(a, workspace, B, c->N);
    hipStream_t st = (hipStream_t)stream;
    if (closed_general(c)) return closed_step_sb(a, workspace, st);
    if (c->N > TRAJ_MAX_N || split_route(c)) return closed_step_long(a, workspace, st);
    const int nr = (B + 63) / 64, nj = (B * c->N + 63) / 64;
    stamp(0, st);
    hipLaunchKernelGGL(rollout_kernel<true>, dim3(nr), dim3(64), 0, st, a);
    stamp(1, st);
    hipLaunchKernelGGL(jac_kernel<true>, dim3(nj), dim3(256), 0, st, a);
    stamp(2, st);
    if (t > 0) {
        // order this step's solves by the previous step's iteration counts (longest first)
        int* perm = (int*)(a.wsWarm + (size_t)B * 4);
        hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, st, (const double*)a.wsWarm, B, perm, 2);
        a.perm = perm;
    }
    stamp(3, st);
    e = launch_mpc(a, st, 2);
    stamp(4, st);
    if ((size_t)(5 * g_ev_used + 4) < g_ev.size()) ++g_ev_used;
    return e;
}

int traj_closed_loop_run(const traj_vehicle_params* p, const traj_mpc_config* c, const traj_paths* paths, int B,
                         double* x, double* u_prev, const double* vref, int t0, int steps, int hist_T,
                         double* hist_x, double* hist_u, int* status, int* iters, void* workspace,
                         size_t workspace_bytes, void* stream) {
    if (!p || B < 0 || steps < 0 || !paths_ok(paths)) return TRAJ_E_ARG;
    int e = check_cfg_closed(c);
    if (e) return e;
    if (B == 0 || steps == 0) return TRAJ_OK;
    if (!x || !u_prev || !vref || t0 < 0) return TRAJ_E_ARG;
    if (!workspace || workspace_bytes < closed_ws_bytes(c, B)) return TRAJ_E_ARG;
    if ((hist_x || hist_u) && t0 + steps > hist_T) return TRAJ_E_ARG;
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    a.p = *p;
    a.c = *c;
    a.B = B;
    a.vref = vref;
    a.path = PathArgs{paths->kmax, paths->kind, paths->pc, paths->nk, paths->xk, paths->coef};
    a.x_state = x;
    a.u_state = u_prev;
    a.t = t0;
    a.hist_T = hist_T;
    a.hist_x = hist_x;
    a.hist_u = hist_u;
    a.status = status;
    a.iters = iters;
    a.dbg = g_dbg;
    a.nsteps = steps;
    a.fused_grid = g_fused_grid;
    // kernel instance: capacity 40, 2 waves per SIMD (3 from TRAJ_FUSED_W3_MIN_STEPS steps when that is set); capacity
    // 80, one wave per SIMD (the lean two-wave instance, traj_debug_fused_waves(2), spills at its 256 registers)
    constexpr int w3_min = TRAJ_FUSED_W3_MIN_STEPS;
    // (by the capacity launch_mpc picks: n = 2N > 40 runs capacity 80 -- 64 only in a TGMPC_CAP64 build, whose fused
    // launch ignores wps -- so 20 < N <= 32 takes the one-wave-per-SIMD instance too; until round 5 it fell through
    // to the opt-in lean two-wave instance, which spills: N = 30 ran 0.68 M against N = 40's 0.99 M)
    a.wps = g_fused_waves ? g_fused_waves : (2 * c->N > 40 ? 1 : ((w3_min > 0 && steps >= w3_min) ? 3 : 2));
    a.spin_limit = g_spin_limit;
    a.dbg_items = g_dbg_items;
    carve_workspace(a, workspace, B, c->N);
    hipStream_t st = (hipStream_t)stream;
    // step queue: [0] next work item, [1] error flag, [2 + b] steps of instance b completed, [2 + B + b] claimed
    a.queue = (int*)(a.wsWarm + (size_t)B * 4) + B;
    if (hipMemsetAsync(a.queue, 0, ((size_t)B * 2 + 2) * sizeof(int), st) != hipSuccess) return TRAJ_E_LAUNCH;
    a.run_ahead = g_run_ahead;
    if (closed_general(c) || (c->N > TRAJ_MAX_N && !split_route(c))) {
        // past the row-split capacity, or with state bounds: the steps as step launch sequences, in order on the
        // stream (the same results as that many traj_closed_loop_step calls; the queue above stays clear, so
        // traj_closed_loop_check reports TRAJ_OK)
        const bool sb = closed_general(c);
        for (int s = 0; s < steps; ++s) {
            KArgs as = a;
            as.t = t0 + s;
            as.status = status ? status + (size_t)s * B : nullptr;
            as.iters = iters ? iters + (size_t)s * B : nullptr;
            as.nsteps = 0;
            e = sb ? closed_step_sb(as, workspace, st) : closed_step_long(as, workspace, st);
            if (e) return e;
        }
        return TRAJ_OK;
    }
    stamp(0, st);
    stamp(1, st);
    stamp(2, st);
    if (t0 == 0) {
        // a run's first launch has no previous order, so order_kernel first runs on the SECOND launch; load
        // its code object now (HIP loads kernels lazily, ~0.75 ms of host time on the first launch) so that
        // cost is not paid inside a later, timed launch
        // (per device: HIP loads code objects per device; one process may drive several GPUs)
        static std::atomic<bool> order_loaded[64];
        int dev = 0;
        if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 && !order_loaded[dev].load()) {
            hipFuncAttributes fa;
            if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&order_kernel)) == hipSuccess)
                order_loaded[dev].store(true);
        }
    }
    if (t0 > 0) {
        // instances ranked by their mean ADMM iterations per step in the previous launch; the kernel
        // pairs ranks heavy-with-light on each workgroup
        int* perm = (int*)(a.wsWarm + (size_t)B * 4);
        hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, st, (const double*)a.wsWarm, B, perm, 3);
        a.perm = perm;
        // heavy instances lead the queue order (mpc_solve.h); none on a first launch (no previous order)
        a.lead_steps = g_lead_steps;
        a.lead_h = (int)(((long long)B * g_lead_permille) / 1000);
        if (a.lead_h >= B) a.lead_h = B - 1;
    }
    stamp(3, st);
    // the row-split kernel's fused instance (the same queue protocol), or the register-resident one
    e = split_route(c) ? launch_split_fused(a, (double*)((char*)workspace + ws_base_bytes(B, c->N)), st)
                       : launch_mpc(a, st, 3);
    stamp(4, st);
    if ((size_t)(5 * g_ev_used + 4) < g_ev.size()) ++g_ev_used;
    return e;
}

int traj_closed_loop_check(const void* workspace, size_t workspace_bytes, int B, int N, void* stream) {
    if (B < 0 || N < 1 || N > TRAJ_MAX_N_GENERAL) return TRAJ_E_ARG;
    if (B == 0) return TRAJ_OK;
    if (!workspace || workspace_bytes < traj_mpc_workspace_bytes(B, N)) return TRAJ_E_ARG;
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    carve_workspace(a, const_cast<void*>(workspace), B, N);
    const int* flag = (const int*)(a.wsWarm + (size_t)B * 4) + B + 1;   // traj_closed_loop_run's queue[1]
    int h = 0;
    hipStream_t st = (hipStream_t)stream;
    if (hipMemcpyAsync(&h, flag, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess) return TRAJ_E_LAUNCH;
    if (hipStreamSynchronize(st) != hipSuccess) return TRAJ_E_LAUNCH;
    return h ? TRAJ_E_HANDOFF : TRAJ_OK;
}

}  // extern "C"
