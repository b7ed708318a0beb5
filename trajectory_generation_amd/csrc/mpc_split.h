// mpc_split.h -- the MPC step with the KKT inverse ROW-SPLIT across lane pairs, register resident: TRAJ_MAX_N < N <=
// TRAJ_MAX_N_SPLIT (n = 2N <= 128 QP variables), no state bounds.
//
// Reference: MPC/mpc_6stati.py:120-275 (mpc_step takes any N, :125) and, CLOSED, one step of MPC/main.py:85-101.  The
// algorithm is the hot kernels' and the long-horizon kernel's (mpc_solve.h, mpc_long.h): the condensed QP over U, box +
// rate rows owned by the variables (A bidiagonal, every product with A or A' a +-2 neighbour exchange), OSQP 0.6's ADMM
// (Ruiz + cost scaling, sigma / alpha, adaptive rho, OSQP termination) and polish (mode 0: OSQP's reduced KKT and
// acceptance rule; mode 1: the exact active-set polish with its KKT certificate), as oracle/ restates them; the KKT
// matrix inverted explicitly by the symmetric sweep operator so that each ADMM iteration is one dense mat-vec.
//
// What changes is where K^-1 lives.  The long-horizon kernel keeps it in LDS (one thread per row, every pivot and every
// mat-vec a read-modify-write of the whole matrix through the LDS pipe, one instance per CU at n > 64).  Here row r of
// K^-1 is held in REGISTERS by two lanes of one wave, lane l and l + 32 (l = r mod 32, wave r / 32): lane half h holds
// columns [h H, h H + H), H = capacity / 2 -- 64 doubles (128 VGPRs) at n = 128, so a row fits beside the solver's state
// in the 256 registers of two waves per SIMD.  The halves are joined by v_permlane32_swap (both lanes then hold the
// same bits: a sum of two partials is commutative), never through LDS:
//   * K^-1 v: each lane forms its half's partial sum (4 FMA chains), one swap, one add;
//   * the sweep's pivot column entry K_rp: the lane half holding column p has it in register 0 (the rows are ROTATED
//     one register per pivot, so the pivot column is always register 0 of its half; after all 2H pivots -- the padding
//     ones are a plain rotation -- the order is the identity again), the other half takes it across the swap;
//   * row maxima (Ruiz norms) and the final sums the same way.
// Per-row scalar state (the ADMM iterate, the scaling, the bounds) is held by both lanes of a row, computed identically.
// The scaled P lives in the caller's scratch (row-major, row r's halves contiguous) and is read for residual checks and
// polish only.  CLOSED: as mpc_long.h (window from the state, warm rho, plant update, history).
#pragma once
#include "mpc_common.h"
#include "mpc_linearize.h"

namespace tgmpc {

// capacities built: H = 40 (n <= 80, 3 waves: rows 80..95 idle), 48 (n <= 96, 3 waves), 64 (n <= 128, 4 waves)
template <int H> struct SplitCfg {
    static constexpr int NR = 2 * H;                 // rows = columns capacity
    static constexpr int WAVES = (NR + 31) / 32;     // 32 rows per wave
    static constexpr int NT = 64 * WAVES;
    static constexpr int NRW = 32 * WAVES;           // row slots (>= NR)
};
__host__ __device__ inline int split_h(int n) { return n <= 80 ? 40 : (n <= 96 ? 48 : 64); }
// per-instance scratch (doubles): the scaled P, NRW rows x 2H
__host__ __device__ inline size_t split_ws_doubles(int N) {
    const int H = split_h(2 * N);
    return (size_t)(32 * ((2 * H + 31) / 32)) * (2 * H);
}

// partner lane's value (lane ^ 32) and the pair sum (the same bits on both lanes)
__device__ __forceinline__ void swap32(double v, double& mine_lo_half, double& mine_hi_half) {
    const int lo = __double2loint(v), hi = __double2hiint(v);
    const auto rl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto rh = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    // after the swap: element 0 holds lanes 0-31 = v[0..31] and lanes 32-63 = v[0..31]; element 1 holds lanes 0-31 =
    // v[32..63] and lanes 32-63 = v[32..63].  So [0] is the half-0 value and [1] the half-1 value of the row, on both.
    mine_lo_half = __hiloint2double(rh[0], rl[0]);
    mine_hi_half = __hiloint2double(rh[1], rl[1]);
}
__device__ __forceinline__ double pair_sum(double v) {
    double a, b;
    swap32(v, a, b);
    return a + b;   // (half 0's partial + half 1's partial, the same operands in the same order on both lanes)
}
__device__ __forceinline__ double pair_max(double v) {   // NaN-propagating
    double a, b;
    swap32(v, a, b);
    return (a > b || a != a) ? a : b;
}

// FUSED (the fused closed loop, traj_closed_loop_run; implies CLOSED): the grid is the resident workgroups, each takes
// (step, instance) work items from the queue in order and waits, if it must, until the instance's previous step is
// complete -- the protocol of mpc_solve.h's fused instances (sc1 state hand-off, the step counter stored after the
// state, the lead set of heavy instances): the linearization runs in the workgroup (block_linearize, stage records in
// LDS) and the P scratch is the workgroup's.  The same values as the per-step launches (rollout_kernel + jac_kernel +
// this kernel), bit for bit.
// INLIN (implied by FUSED; the step entry point's default, traj_debug_step_linearize): the same in-workgroup
// linearization for a step launch -- one launch per call instead of rollout_kernel + jac_kernel + this kernel, the
// drop-in call's latency; bit-identical to the three-launch sequence.
#ifndef TGMPC_SPLIT_GHOST
#define TGMPC_SPLIT_GHOST 1
#endif
constexpr bool SPLIT_GHOST = TGMPC_SPLIT_GHOST != 0;
#ifndef TGMPC_SPLIT_BLOCK
// pivots per sweep round: 2 (one LDS round and one barrier per pair; the default) or 1 (the single sweep).  A 4-pivot
// form (a per-lane LDL' solve of the block) measured 1.34-1.37 M against 1.42 M at config 3 and moved one capped
// instance's status in test_config3_iteration_cap_steps_vs_oracle; it is not kept
#define TGMPC_SPLIT_BLOCK 2
#endif
constexpr int SPLIT_BLOCK = TGMPC_SPLIT_BLOCK;
constexpr bool SPLIT_BLOCK2 = SPLIT_BLOCK == 2;
static_assert(SPLIT_BLOCK == 1 || SPLIT_BLOCK == 2, "sweep block");
#ifndef TGMPC_SPLIT_NOZERO_TIMING
#define TGMPC_SPLIT_NOZERO_TIMING 0   // 1: timing experiment only (wrong results): the pivot rows are not zeroed
#endif
// DIAG (fused only, when a diagnostic buffer is set: traj_debug_set_stamps): per-phase s_memtime stamps of each
// instance's last step in a.dbg[b][0..11] (tools/split_phase.py); the production instances compile none of it.
template <int H, bool CLOSED = false, bool FUSED = false, bool INLIN = FUSED, bool DIAG = false>
__global__ __launch_bounds__(SplitCfg<H>::NT) __attribute__((amdgpu_waves_per_eu(2))) void solve_split_kernel(
    const KArgs a0, double* sws, size_t sstride) {
    static_assert(!FUSED || CLOSED, "the fused run is the closed loop");
    static_assert(!FUSED || INLIN, "the fused run linearizes in the workgroup");
    using SC = SplitCfg<H>;
    constexpr int NR = SC::NR, NT = SC::NT, NRW = SC::NRW, WAVES = SC::WAVES;
    constexpr int PL = 2 * H;                 // P row stride (doubles)
    constexpr int SPV = 2 * H + 2;            // one pivot-row slice buffer: [off + m], m < 2H, off in {0, 1}
    __shared__ __attribute__((aligned(16))) double s_bc[2][NRW];       // broadcast vectors (rotating)
    __shared__ double s_ex[4][NRW];                                    // +-2 exchanges (rotating)
    // ADMM: every row's constants of the rate-row update, read by the row two below it (the ghost update, below)
    __shared__ __attribute__((aligned(16))) double s_gh[SPLIT_GHOST ? NRW + 2 : 1][6];
    __shared__ __attribute__((aligned(16))) double s_pv[SPLIT_BLOCK > 1 ? 1 : 2][2][SPV];   // sweep: [parity][half][slice]
    // block sweep: [parity][column of the block][half][slice]
    __shared__ __attribute__((aligned(16))) double s_pv2[SPLIT_BLOCK2 ? 2 : 1][SPLIT_BLOCK2 ? 2 : 1][2][SPV];
    __shared__ double s_red[WAVES * 8];
    __shared__ int s_flag[4];
    __shared__ double s_xc[CLOSED || INLIN ? 6 : 1], s_uc[CLOSED || INLIN ? 2 : 1];
    __shared__ double s_prc[CLOSED ? 3 * (NR / 2 + 1) : 1];
    __shared__ double s_xs[6 * (NR / 2 + 1)];                          // outputs: X by the linear model
    __shared__ double s_vr[NR / 2 + 1], s_sc[NR / 2 + 1][2];          // vref_k; sin / cos of the window's phi*_k
    // One LDS region for the condensing phase's buffers -- F_k rows of a block of stages, INLIN's stage records -- and,
    // PLDS (the closed loop at H = 40), the scaled P after it (NR rows, stride PS): otherwise P lives in the caller's
    // scratch, where its re-reads (each factorization, each residual check, the polish) went to HBM
    constexpr bool PLDS = CLOSED && H == 40;
    constexpr int PS = PLDS ? PL + 2 : PL;   // P row stride (LDS: padded against bank conflicts)
    constexpr int UN_COND = 8 * 3 * NRW + (INLIN ? LREC * (NR / 2) : 2), UN_P = PLDS ? NR * PS : 0;
    __shared__ __attribute__((aligned(16))) double s_un[UN_COND > UN_P ? UN_COND : UN_P];
    double(*const s_Fb)[3][NRW] = reinterpret_cast<double(*)[3][NRW]>(s_un);   // condensing: [stage in block][F row]
    double* const s_rec = s_un + 8 * 3 * NRW;                                     // INLIN: the stage records
    __shared__ int s_item;
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    const int r = 32 * wid + (lane & 31), h = lane >> 5;    // row, half
    // the P scratch: per instance (one workgroup per instance), or per workgroup (fused: a workgroup solves one item
    // at a time)
    double* const Pg = sws + (size_t)blockIdx.x * sstride;   // scaled P, row r at Pg + r PL (!PLDS)
    // row rr_ of the scaled P (PLDS: lanes past NR -- padding, never read by a real row -- alias rows below NR)
    auto Prow = [&](int rr_) -> double* {
        return PLDS ? s_un + (size_t)(rr_ < NR ? rr_ : rr_ - NR) * PS : Pg + (size_t)rr_ * PL;
    };
    for (bool more = true; more;) {
    more = FUSED;
    // fused: the arguments through a pointer the compiler cannot see through, so that nothing derived from them is
    // hoisted out of the item loop (it would stay live across every solve and spill) -- mpc_solve.h's device
    typedef __attribute__((address_space(4))) const KArgs* KArgsPtr;
    KArgsPtr ap = FUSED ? (KArgsPtr)__builtin_amdgcn_kernarg_segment_ptr() : (KArgsPtr) nullptr;
    if constexpr (FUSED) asm volatile("" : "+s"(ap));
    const KArgs& a = FUSED ? *(const KArgs*)ap : a0;
    int b = blockIdx.x, step = 0;
    if constexpr (FUSED) {
        // item q <-> (step, rank) in the queue order of mpc_solve.h: the heavy ranks' first lead steps, then level s =
        // the heavy ranks' step s + lead and the light ranks' step s; an item only ever waits for one drawn before it
        const int Bq = a.B, S = a.nsteps;
        const int L = (a.lead_h > 0) ? min(a.lead_steps, S) : 0, Hh = (L > 0) ? a.lead_h : 0;
        const int P0 = L * Hh, full = (S - L) * Bq;
        __syncthreads();
        if (t == 0) s_item = atomicAdd(&a.queue[0], 1);
        __syncthreads();
        const int q = s_item;
        if (q >= Bq * S) break;
        int rank;
        if (q < P0) {
            step = q / Hh;
            rank = q - step * Hh;
        } else if (q - P0 < full) {
            const int lv = (q - P0) / Bq;
            rank = (q - P0) - lv * Bq;
            step = (rank < Hh) ? lv + L : lv;
        } else {
            const int q2 = q - P0 - full, lv = (S - L) + q2 / (Bq - Hh);
            rank = Hh + (q2 - (lv - (S - L)) * (Bq - Hh));
            step = lv;
        }
        b = a.perm ? a.perm[rank] : rank;
        if (t == 0 && step > 0) {
            int spins = 0;
            while (__hip_atomic_load(&a.queue[2 + b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < step) {
                __builtin_amdgcn_s_sleep(2);
                if (++spins > a.spin_limit) {   // bounded: a lost hand-off is reported (TRAJ_E_HANDOFF), never a hang
                    __hip_atomic_store(&a.queue[1], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
    }
    const int tstep = a.t + step;
    // diagnostics: slot i of this instance's record, written by thread 0 at the launch's last step (DIAG only)
    long long* const dbg = (DIAG && t == 0 && (!FUSED || step == a.nsteps - 1)) ? a.dbg : nullptr;
    auto stamp = [&](int i, long long v) {
        if (DIAG && dbg) dbg[(size_t)b * 32 + i] = v;
    };
    [[maybe_unused]] long long cyc_sweep = 0, cyc_pol = 0, t_prev = 0, cyc_swb = 0, cyc_xb = 0, cyc_sw1 = 0, cyc_sw2 = 0;
    [[maybe_unused]] int n_fact = 0, ph_prev = -1;
    stamp(0, __builtin_amdgcn_s_memtime());
    const traj_vehicle_params& p = a.p;
    const traj_mpc_config& c = a.c;
    const int N = c.N, n = 2 * N;
    const bool own = r < n;
    const int kk = r >> 1, ch = r & 1;
    const double* vr = a.vref + (size_t)(N + 1) * b;

    // ---- block helpers ----
    int xb = 0, bb = 0;
    auto exch = [&](double v, int delta) -> double {   // value of row r + delta (0 outside 0..n-1)
        double* buf = s_ex[xb & 3];
        xb++;
        if (h == 0) buf[r] = v;
        [[maybe_unused]] long long tb0 = 0;
        if constexpr (DIAG) tb0 = __builtin_amdgcn_s_memtime();
        __syncthreads();
        if constexpr (DIAG) cyc_xb += (long long)__builtin_amdgcn_s_memtime() - tb0;
        const int s = r + delta;
        return (own && s >= 0 && s < n) ? buf[s] : 0.0;
    };
    // two exchanges in one round (one barrier): the values of rows r + d1 and r + d2
    auto exch2 = [&](double v1, int d1, double v2, int d2, double& o1, double& o2) {
        double* buf1 = s_ex[xb & 3];
        double* buf2 = s_ex[(xb + 1) & 3];
        xb += 2;
        if (h == 0) {
            buf1[r] = v1;
            buf2[r] = v2;
        }
        __syncthreads();
        const int s1 = r + d1, s2 = r + d2;
        o1 = (own && s1 >= 0 && s1 < n) ? buf1[s1] : 0.0;
        o2 = (own && s2 >= 0 && s2 < n) ? buf2[s2] : 0.0;
    };
    auto bcast = [&](double v) -> const double* {
        double* buf = s_bc[bb & 1];
        bb++;
        if (h == 0) buf[r] = own ? v : 0.0;
        [[maybe_unused]] long long tb0 = 0;
        if constexpr (DIAG) tb0 = __builtin_amdgcn_s_memtime();
        __syncthreads();
        if constexpr (DIAG) cyc_xb += (long long)__builtin_amdgcn_s_memtime() - tb0;
        return buf;
    };
    // Block reductions over DPP (wave_max_dpp / wave_sum_dpp: no per-lane shuffle addresses, which the compiler would
    // hoist out of the solver's loops and keep live -- spilled -- across the whole solve), then the waves in order.
    // block max of V values >= 0, NaN propagating (uniform; both halves hold the same per-row values, duplicates are
    // harmless in a max)
    auto nmax = [](double x_, double y_) { return (x_ > y_ || x_ != x_) ? x_ : y_; };
    auto block_max = [&](auto& v) {
        constexpr int V = sizeof(v) / sizeof(double);
        static_assert(V <= 8, "s_red");
        wave_max_dpp<V>(v);
        if (lane == 0) {
#pragma unroll
            for (int i = 0; i < V; ++i) s_red[wid * 8 + i] = v[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < V; ++i) {
            double m = s_red[i];
            for (int w = 1; w < WAVES; ++w) m = nmax(m, s_red[w * 8 + i]);
            v[i] = m;
        }
        __syncthreads();
    };
    // block sum of sv over the rows (half-0 lanes: the DPP pattern per wave, then the waves in order) and block max of
    // mv, in one round
    auto block_sum_max = [&](double sv, double mv, double& so, double& mo) {
        sv = wave_sum_dpp((h == 0) ? sv : 0.0);
        double m1[1] = {mv};
        wave_max_dpp<1>(m1);
        if (lane == 0) {
            s_red[wid * 8] = sv;
            s_red[wid * 8 + 1] = m1[0];
        }
        __syncthreads();
        double sacc = 0.0;
        for (int w = 0; w < WAVES; ++w) sacc += s_red[w * 8];
        double m = s_red[1];
        for (int w = 1; w < WAVES; ++w) m = nmax(m, s_red[w * 8 + 1]);
        __syncthreads();
        so = sacc;
        mo = m;
    };

    // ---- inputs (:144-163 normalisation by the caller; CLOSED: state, u_prev and the window) ----
    if constexpr (CLOSED) {
        if (FUSED) {   // the state the instance's previous step published (sc1 loads, mpc_solve.h st_coh / ld_coh)
            if (t < 6) s_xc[t] = ld_coh(a.x_state + 6 * (size_t)b + t);
            if (t < 2) s_uc[t] = ld_coh(a.u_state + 2 * (size_t)b + t);
        } else {
            if (t < 6) s_xc[t] = a.x_state[6 * (size_t)b + t];
            if (t < 2) s_uc[t] = a.u_state[2 * (size_t)b + t];
        }
        __syncthreads();
        if (t == 0) {   // main.py:51-68: xs_{k+1} = xs_k + vref_k Ts (serial, as ref_window_kernel)
            double xs = s_xc[0];
            s_prc[0] = xs;
            for (int k = 0; k < N; ++k) {
                xs = xs + vr[k] * c.Ts;
                s_prc[3 * (k + 1)] = xs;
            }
        }
        __syncthreads();
        for (int k = t; k <= N; k += NT) {
            double y, dy;
            path_eval(a.path, b, s_prc[3 * k], y, dy);
            s_prc[3 * k + 1] = y;
            const double ph = pm_atan(dy);
            s_prc[3 * k + 2] = ph;
            pm_sincos(ph, &s_sc[k][0], &s_sc[k][1]);
        }
    }
    if constexpr (INLIN && !CLOSED) {   // the step's state and input, staged for block_linearize
        if (t < 6) s_xc[t] = a.x0[6 * (size_t)b + t];
        if (t < 2) s_uc[t] = a.u_prev[2 * (size_t)b + t];
    }
    const double* x0 = (CLOSED || INLIN) ? s_xc : a.x0 + 6 * (size_t)b;
    const double* up = (CLOSED || INLIN) ? s_uc : a.u_prev + 2 * (size_t)b;
    const double* pref = CLOSED ? s_prc : a.path_ref + (size_t)3 * (N + 1) * b;
    // the stage loops' per-stage inputs that do not depend on the chain, in LDS before it starts: vref_k, and sin / cos
    // of phi*_k (one stage per thread, the same calls as in the loop)
    for (int k = t; k <= N; k += NT) {
        s_vr[k] = vr[k];
        if constexpr (!CLOSED) pm_sincos(pref[3 * k + 2], &s_sc[k][0], &s_sc[k][1]);
    }
    if (t == 0) { s_flag[0] = 0; s_flag[1] = 0; }
    __syncthreads();
    // A_k, B_k, g_k: the workspace's (stage k at gA + RA k, ...), or, fused, the stage records the workgroup's own
    // linearization leaves in LDS (block_linearize: rollout_kernel + jac_kernel's values, bit for bit)
    stamp(1, __builtin_amdgcn_s_memtime());
    if constexpr (INLIN) block_linearize<NT>(t, p, N, c.Ts, s_xc, s_uc, s_rec, nullptr);
    stamp(2, __builtin_amdgcn_s_memtime());
    constexpr int RA = INLIN ? LREC : 36, RB = INLIN ? LREC : 12, RG = INLIN ? LREC : 6;
    const double* gA = INLIN ? s_rec : a.Ad + (size_t)36 * N * b;
    const double* gB = INLIN ? s_rec + 36 : a.Bd + (size_t)12 * N * b;
    const double* gg = INLIN ? s_rec + 48 : a.gd + (size_t)6 * N * b;
    {
        int bad = 0;
        if (t < 6) bad |= !isfinite(x0[t]);
        if (t < 2) bad |= !isfinite(up[t]);
        for (int i = t; i < 3 * (N + 1); i += NT) bad |= !isfinite(pref[i]);
        for (int i = t; i < N + 1; i += NT) bad |= !isfinite(vr[i]);
        if (bad) s_flag[0] = 1;
    }

    // ---- condensed QP (:180-250): P = sum_k F_k' F_k (+ the input penalties), q ----
    // row r carries column r of the input sensitivity G_k; the free response xh is uniform.  Lane half h accumulates
    // columns [h H, h H + H) of row r: Ph[i] = P_{r, h H + i}.
    const double sw0 = sqrt(2.0 * c.q_c), sw1 = sqrt(2.0 * c.q_phi), sw2 = sqrt(2.0 * c.q_vx);
    double xh[6], G[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 6; ++i) xh[i] = x0[i];
    double qi = 0.0;
    double Kh[H];   // row r, columns of half h: P after condensing, through scaling, then K and K^-1
    // The stages in blocks of KB: first the block's sensitivities -- G_k, the free response, F_k (3 values of row r per
    // stage, published to LDS) and q -- then the block's products on the matrix cores: P = sum_k F_k' F_k as 16 x 16
    // tiles of the upper triangle, one v_mfma_f64_16x16x4f64 per tile and stage (k-rows = F_k's rows, one zero), the
    // tiles dealt round-robin to the waves (accumulators in registers for the whole stage loop).  Each unordered
    // pair of columns is formed by one accumulation, so P is exactly symmetric; F_k's columns >= 2 (k + 1) are zero
    // (inputs of later stages), so a tile whose column block starts there adds +-0 and is skipped.  The tiles then go
    // to the P scratch (both triangles), from which each lane loads its half-row.
    constexpr int KB = 8;
    // Row rr of A_k x (+ v) as the chain v = fma(A[rr][cc], x[cc], v), cc = 0..5.  CLOSED: A_k comes from the library's
    // own linearization, whose structural entries are exact (f does not read X, Y; f_0, f_1 do not read omega;
    // f_2 = omega; f_3..5 do not read phi: rows 0 / 1 = [1 0 a a a 0], row 2 = [0 0 1 0 0 a], rows 3..5 =
    // [0 0 0 a a a]), so the chain skips the zero terms and adds the unit ones -- the values of the full chain (up to
    // the sign of a zero), as mpc_solve.h's capacity kernels form them; the step entry point keeps the full chain.
    auto arow = [&](const double* Ak, int rr, const double* x, double v) -> double {
        if constexpr (CLOSED) {
            if (rr <= 1) {
                v = v + x[rr];
#pragma unroll
                for (int cc = 2; cc < 5; ++cc) v = fma(Ak[6 * rr + cc], x[cc], v);
            } else if (rr == 2) {
                v = v + x[2];
                v = fma(Ak[6 * 2 + 5], x[5], v);
            } else {
#pragma unroll
                for (int cc = 3; cc < 6; ++cc) v = fma(Ak[6 * rr + cc], x[cc], v);
            }
        } else {
#pragma unroll
            for (int cc = 0; cc < 6; ++cc) v = fma(Ak[6 * rr + cc], x[cc], v);
        }
        return v;
    };
    constexpr int NB = NR / 16;                   // 16-wide column blocks
    constexpr int NTILE = NB * (NB + 1) / 2;
    constexpr int MT = (NTILE + WAVES - 1) / WAVES;   // tiles per wave
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = d4{0.0, 0.0, 0.0, 0.0};
    // MFMA operand slot of this lane: k-row, column (from an opaque copy of the lane index: in the fused item loop the
    // derived LDS / scratch addresses would otherwise be hoisted out of it and kept live across the whole solve)
    int lane_o = lane;
    asm volatile("" : "+v"(lane_o));
    const int mr = (lane_o >> 4) & 3, mc = lane_o & 15;
    // the F row in MFMA k-slot mr: F2, F1, F0, then the zero row.  v_mfma_f64_16x16x4f64 accumulates its four k-slots
    // as one fma each, in slot order (measured: tools/split_bitcmp.py), so each entry is fma(F0, ., fma(F1, ., fma(F2,
    // ., acc))) -- the per-lane FMA chain of the row form, bit for bit (the other slot orders differ in the last bits)
    const int fk = mr < 3 ? 2 - mr : -1;
    [[maybe_unused]] long long cyc_c1 = 0, cyc_c2 = 0, cyc_cb = 0, tc = 0;   // DIAG: condensing sub-phases
    for (int k0 = 0; k0 < N; k0 += KB) {
        const int kend = (k0 + KB < N) ? k0 + KB : N;
        if constexpr (DIAG) tc = __builtin_amdgcn_s_memtime();
        for (int k = k0; k < kend; ++k) {
            const double* Ak = gA + RA * k;
            double xn[6], Gn[6];
            for (int rr = 0; rr < 6; ++rr) {
                xn[rr] = arow(Ak, rr, xh, gg[RG * k + rr]);
                const double w = arow(Ak, rr, G, 0.0);
                Gn[rr] = (own && kk == k) ? gB[RB * k + 2 * rr + ch] : w;
            }
            for (int rr = 0; rr < 6; ++rr) { xh[rr] = xn[rr]; G[rr] = Gn[rr]; }
            const int k1 = k + 1;
            const double sk = s_sc[k1][0], ck = s_sc[k1][1];
            const double e0 = sk * (xh[0] - pref[3 * k1]) - ck * (xh[1] - pref[3 * k1 + 1]);
            const double e1 = xh[2] - pref[3 * k1 + 2];
            const double e2 = xh[3] - s_vr[k1];
            const double F0 = sw0 * (sk * G[0] - ck * G[1]), F1 = sw1 * G[2], F2 = sw2 * G[3];
            qi += sw0 * F0 * e0 + sw1 * F1 * e1 + sw2 * F2 * e2;
            if (h == 0) {
                s_Fb[k - k0][0][r] = F0;
                s_Fb[k - k0][1][r] = F1;
                s_Fb[k - k0][2][r] = F2;
            }
        }
        if constexpr (DIAG) {
            const long long now = __builtin_amdgcn_s_memtime();
            cyc_c1 += now - tc;
            tc = now;
        }
        __syncthreads();
        if constexpr (DIAG) {
            const long long now = __builtin_amdgcn_s_memtime();
            cyc_cb += now - tc;
            tc = now;
        }
        for (int k = k0; k < kend; ++k) {
            double opv[NB];   // this lane's operand slot of each column block: F_k[mr][16 ib + mc] (row 3: 0)
#pragma unroll
            for (int ib = 0; ib < NB; ++ib) opv[ib] = (fk >= 0) ? s_Fb[k - k0][fk >= 0 ? fk : 0][16 * ib + mc] : 0.0;
            int ti = 0;
#pragma unroll
            for (int ib = 0; ib < NB; ++ib)
#pragma unroll
                for (int jb = ib; jb < NB; ++jb, ++ti)
                    if (ti % WAVES == wid && 16 * jb < 2 * k + 2)
                        acc[ti / WAVES] = __builtin_amdgcn_mfma_f64_16x16x4f64(opv[ib], opv[jb], acc[ti / WAVES], 0, 0, 0);
        }
        if constexpr (DIAG) {
            const long long now = __builtin_amdgcn_s_memtime();
            cyc_c2 += now - tc;
            tc = now;
        }
        __syncthreads();
        if constexpr (DIAG) cyc_cb += (long long)__builtin_amdgcn_s_memtime() - tc;
    }
    {   // the tiles to the P scratch (accumulator lane: row 16 ib + mr + 4 reg, column 16 jb + mc), both triangles;
        // the scratch rows past NR (padding lanes' rows) are zeroed by their lanes
        int ti = 0;
#pragma unroll
        for (int ib = 0; ib < NB; ++ib)
#pragma unroll
            for (int jb = ib; jb < NB; ++jb, ++ti)
                if (ti % WAVES == wid) {
#pragma unroll
                    for (int reg = 0; reg < 4; ++reg) {
                        const int i = 16 * ib + mr + 4 * reg, j = 16 * jb + mc;
                        const double v = acc[ti / WAVES][reg];
                        Prow(i)[j] = v;
                        if (ib != jb) Prow(j)[i] = v;
                    }
                }
        if constexpr (NRW > NR && !PLDS) {
            if (r >= NR) {
                double2* w2 = reinterpret_cast<double2*>(Pg + (size_t)r * PL + h * H);
#pragma unroll
                for (int i = 0; i < H; i += 2) w2[i / 2] = double2{0.0, 0.0};
            }
        }
    }
    __syncthreads();
    stamp(12, cyc_c1);
    stamp(13, cyc_c2);
    stamp(14, cyc_cb);
    // input penalties U'RU and dU'Rd dU (dU_0 = U_0 - u_prev): the band of row r
    double Rs[4], Rds[4];
    Rs[0] = c.R[0]; Rs[3] = c.R[3]; Rs[1] = Rs[2] = 0.5 * (c.R[1] + c.R[2]);
    Rds[0] = c.Rd[0]; Rds[3] = c.Rd[3]; Rds[1] = Rds[2] = 0.5 * (c.Rd[1] + c.Rd[2]);
    const double Rs0 = ch ? Rs[2] : Rs[0], Rs1 = ch ? Rs[3] : Rs[1];
    const double Rd0 = ch ? Rds[2] : Rds[0], Rd1 = ch ? Rds[3] : Rds[1];
    if (own) {
        // row r's band entries (columns 2 kk - 2 .. 2 kk + 3) in the scratch, by the half-0 lane (dynamic columns: no
        // per-register selects), then both halves reload the row
        if (h == 0) {
            // (from an opaque copy of the row index: the band's row address, formed once outside the fused item loop,
            // would stay live across it and spill)
            int r_o = r;
            asm volatile("" : "+v"(r_o));
            const int kk_o = r_o >> 1;
            const double dmul = (kk_o < N - 1) ? 2.0 : 1.0;
            double* const pr_ = Prow(r_o);
            const int j0 = 2 * kk_o - 2 > 0 ? 2 * kk_o - 2 : 0, j1 = 2 * kk_o + 4 < n ? 2 * kk_o + 4 : n;
            for (int j = j0; j < j1; ++j) {
                const int kj = j >> 1;
                const double rs = (j & 1) ? Rs1 : Rs0, rd = (j & 1) ? Rd1 : Rd0;
                const double add = (kj == kk_o) ? 2.0 * rs + 2.0 * rd * dmul : -2.0 * rd;
                pr_[j] = pr_[j] + add;
            }
        }
        if (kk == 0) qi -= 2.0 * (Rd0 * up[0] + Rd1 * up[1]);
    }
    __syncthreads();
    {
        double* pp = Prow(r) + h * H;   // this lane's half-row
        asm volatile("" : "+v"(pp));
        const double2* pp2 = reinterpret_cast<const double2*>(pp);
#pragma unroll
        for (int i = 0; i < H; i += 2) {
            const double2 v2 = pp2[i / 2];
            Kh[i] = v2.x;
            Kh[i + 1] = v2.y;
        }
    }
    // row maximum |P_rj| (both halves)
    auto row_absmax = [&]() -> double {
        double m4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int i = 0; i < H; ++i) m4[i & 3] = vmax_abs(m4[i & 3], Kh[i]);
        return pair_max(vmax(vmax(m4[0], m4[1]), vmax(m4[2], m4[3])));
    };
    // constraint rows owned by r: box (U_r) and rate (U_r - U_{r-2}, or U_0 - u_prev)
    double lb = ch ? c.u_lo[1] : c.u_lo[0], ub = ch ? c.u_hi[1] : c.u_hi[0];
    double lr = ch ? c.du_lo[1] : c.du_lo[0], ur = ch ? c.du_hi[1] : c.du_hi[0];
    if (kk == 0) { lr += up[ch]; ur += up[ch]; }
    const bool has_prev = kk > 0;
    {
        // (a NaN entry: the max propagates it; an infinite one is caught as non-finite)
        const double am = row_absmax();
        int bad = 0;
        if (own) bad |= !isfinite(qi) || !isfinite(am);
        if (bad) s_flag[0] = 1;
    }
    // exact feasibility of the box + rate chain (interval propagation)
    if (t < 2) {
        double lo = up[t], hi = up[t];
        const double dlo = t ? c.du_lo[1] : c.du_lo[0], dhi = t ? c.du_hi[1] : c.du_hi[0];
        const double ulo = t ? c.u_lo[1] : c.u_lo[0], uhi = t ? c.u_hi[1] : c.u_hi[0];
        for (int k = 0; k < N; ++k) {
            double nlo = lo + dlo, nhi = hi + dhi;
            if (nlo < ulo) nlo = ulo;
            if (nhi > uhi) nhi = uhi;
            if (!(nlo <= nhi)) s_flag[1] = 1;
            lo = nlo;
            hi = nhi;
        }
    }
    __syncthreads();
    const int early = s_flag[0] ? TRAJ_STATUS_SOLVER_ERROR : (s_flag[1] ? TRAJ_STATUS_INFEASIBLE : -1);
    stamp(3, __builtin_amdgcn_s_memtime());
    int status = TRAJ_STATUS_SOLVER_ERROR, iter = 0, pol = 0;
    double xsol = 0.0;

    if (early < 0) {
        // ---- Ruiz equilibration + cost scaling (OSQP scale_data), as mpc_solve.h / mpc_long.h ----
        double D = 1.0, Eb = 1.0, Er = 1.0, cs = 1.0, cn = 0.0;
        cn = own ? row_absmax() : 0.0;
        for (int it = 0; it < c.scaling_iters; ++it) {
            double Er_up, D_dn;
            exch2(Er, +2, D, -2, Er_up, D_dn);
            const double a_b = Eb * D, a_r = Er * D, a_rm = has_prev ? Er * D_dn : 0.0, a_rp = Er_up * D;
            const double pn = cs * cn;
            const double coln = fmax(pn, fmax(fmax(fabs(a_b), fabs(a_r)), fabs(a_rp)));
            const double Dt = own ? 1.0 / sqrt(limit_scaling(coln)) : 1.0;
            const double Etb = 1.0 / sqrt(limit_scaling(fabs(a_b)));
            const double Etr = 1.0 / sqrt(limit_scaling(fmax(fabs(a_r), fabs(a_rm))));
            const double* dv = bcast(Dt);
            double m4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int i = 0; i < H; ++i) {
                const double w = Kh[i] * (Dt * dv[h * H + i]);
                Kh[i] = w;
                m4[i & 3] = vmax_abs(m4[i & 3], w);
            }
            cn = own ? pair_max(vmax(vmax(m4[0], m4[1]), vmax(m4[2], m4[3]))) : 0.0;
            qi *= Dt;
            D *= Dt;
            Eb *= Etb;
            Er *= Etr;
            double csum, qmax;
            block_sum_max(own ? cs * cn : 0.0, own ? fabs(cs * qi) : 0.0, csum, qmax);
            const double mean = csum / n;
            double ct = fmax(mean, limit_scaling(qmax));
            ct = 1.0 / limit_scaling(ct);
            cs *= ct;
        }
#pragma unroll
        for (int i = 0; i < H; ++i) Kh[i] *= cs;
        qi *= cs;
        // the scaled P to the scratch (row r's half h at Pg + r PL + h H); the padding rows r >= n hold the identity
        // row there (zero otherwise), so that K's padding pivots are trivial
        {   // (the scratch holds NRW rows: padding rows past NR park there too, never read by a real row; PLDS: they
            // do not store)
            if (!PLDS || r < NR) {
                double2* w2 = reinterpret_cast<double2*>(Prow(r) + h * H);
#pragma unroll
                for (int i = 0; i < H; i += 2) w2[i / 2] = double2{Kh[i], Kh[i + 1]};
            }
            if (!own && r < NR && h == r / H) Prow(r)[r] = 1.0;
        }
        const double csinv = 1.0 / cs;
        const double D_dn = exch(D, -2);
        const double a_b = Eb * D, a_r = Er * D, a_rm = has_prev ? Er * D_dn : 0.0;
        const double a_r_up = exch(a_r, +2);
        const double slb = (lb > -INFTY) ? lb * Eb : -INFTY, sub = (ub < INFTY) ? ub * Eb : INFTY;
        const double slr = (lr > -INFTY) ? lr * Er : -INFTY, sur = (ur < INFTY) ? ur * Er : INFTY;
        const double Dinv = 1.0 / D, Ebinv = 1.0 / Eb, Erinv = 1.0 / Er;
        __syncthreads();   // P in the scratch (read back by other lanes' row loads only through the same lane: no hazard)

        // ---- helpers over the scaled problem ----
        auto Ax = [&](double v, double& zb, double& zr) {
            const double vdn = exch(v, -2);
            zb = a_b * v;
            zr = a_r * v - a_rm * vdn;
        };
        auto ATw = [&](double wb, double wr) -> double {
            const double rp_up = exch(a_rm * wr, +2);   // a_rp(r) wr(r+2), formed on row r+2
            return a_b * wb + a_r * wr - rp_up;
        };
        // (P v)_r: the half-row from the scratch (16-byte loads, all in flight), 4 chains, the pair sum
        auto Pmul = [&](double v) -> double {
            const double* vb = bcast(v);
            const double2* v2 = reinterpret_cast<const double2*>(__builtin_assume_aligned(vb + h * H, 16));
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
            const double2* p2 = reinterpret_cast<const double2*>(Prow(r) + h * H);
#pragma unroll
            for (int i0 = 0; i0 < H; i0 += 8) {
                double2 pv[4], vv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) { pv[i] = p2[i0 / 2 + i]; vv[i] = v2[i0 / 2 + i]; }
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    s4[(2 * i) & 3] = fma(pv[i].x, vv[i].x, s4[(2 * i) & 3]);
                    s4[(2 * i + 1) & 3] = fma(pv[i].y, vv[i].y, s4[(2 * i + 1) & 3]);
                }
            }
            const double s = pair_sum((s4[0] + s4[1]) + (s4[2] + s4[3]));
            return own ? s : 0.0;
        };
        // (K^-1 v)_r from the register half-rows: the broadcast half in chunks of 8 (16-byte reads), 4 chains
        auto Kmul = [&](double v) -> double {
            const double* vb = bcast(v);
            const double2* v2 = reinterpret_cast<const double2*>(__builtin_assume_aligned(vb + h * H, 16));
            double s4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int i0 = 0; i0 < H; i0 += 8) {
                double2 vv[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) vv[i] = v2[i0 / 2 + i];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    s4[(i0 + 2 * i) & 3] = fma(Kh[i0 + 2 * i], vv[i].x, s4[(i0 + 2 * i) & 3]);
                    s4[(i0 + 2 * i + 1) & 3] = fma(Kh[i0 + 2 * i + 1], vv[i].y, s4[(i0 + 2 * i + 1) & 3]);
                }
            }
            const double s = pair_sum((s4[0] + s4[1]) + (s4[2] + s4[3]));
            return own ? s : 0.0;
        };
        auto rho_for = [&](double l, double u, double rho) -> double {
            if (l <= -INFTY * MIN_SCALING && u >= INFTY * MIN_SCALING) return RHO_MIN;
            if (u - l < RHO_TOL) return RHO_EQ_OVER_INEQ * rho;
            return rho;
        };
        struct Res { double pr, dr, eps_p, eps_d, prs, drs, pn, dn; };
        auto residuals = [&](double x, double zb, double zr, double yb, double yr) -> Res {
            const double px = Pmul(x);
            double axb, axr;
            Ax(x, axb, axr);
            const double aty = ATw(yb, yr);
            double v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (own) {
                const double dres = px + qi + aty;
                v[0] = fmax(fabs(Ebinv * (axb - zb)), fabs(Erinv * (axr - zr)));
                v[1] = fmax(fmax(fabs(Ebinv * axb), fabs(Erinv * axr)), fmax(fabs(Ebinv * zb), fabs(Erinv * zr)));
                v[2] = fabs(Dinv * dres) * csinv;
                v[3] = fmax(fabs(Dinv * px) * csinv, fmax(fabs(Dinv * aty) * csinv, fabs(Dinv * qi) * csinv));
                v[4] = fmax(fabs(axb - zb), fabs(axr - zr));
                v[5] = fabs(dres);
                v[6] = fmax(fmax(fabs(axb), fabs(axr)), fmax(fabs(zb), fabs(zr)));
                v[7] = fmax(fmax(fabs(aty), fabs(qi)), fabs(px));
            }
            block_max(v);
            Res rs;
            rs.pr = v[0]; rs.eps_p = c.eps_abs + c.eps_rel * v[1];
            rs.dr = v[2]; rs.eps_d = c.eps_abs + c.eps_rel * v[3];
            rs.prs = v[4]; rs.drs = v[5]; rs.pn = v[6]; rs.dn = v[7];
            return rs;
        };

        // ---- ADMM (osqp_solve) + polish around one factorization site ----
        constexpr int PH_ADMM = 0, PH_POLISH = 1, PH_DONE = 2;
        int phase = PH_ADMM;
        double rho = c.rho;
        if (CLOSED && c.warm_start && tstep > 0 && a.wsWarm) {   // closed-loop warm start: the previous step's rho
            const double* wv = a.wsWarm + 4 * (size_t)b;
            const double w0 = FUSED ? ld_coh(wv) : wv[0], w1 = FUSED ? ld_coh(wv + 1) : wv[1];
            if (w1 != 0.0) rho = fmin(fmax(w0, RHO_MIN), RHO_MAX);
        }
        double x = 0.0, zb = 0.0, zr = 0.0, yb = 0.0, yr = 0.0;
        double zr_g = 0.0, yr_g = 0.0;   // the ghost of row r + 2's rate-row state (SPLIT_GHOST)
        double rb = rho_for(slb, sub, rho), rr = rho_for(slr, sur, rho);
        Res rs0 = {0, 0, 0, 0, 0, 0, 0, 0};
        int rounds = 0, ps = 0, actb = 0, actr = 0;
        double escale = 1.0;
        const double alpha = c.alpha, sig = c.sigma, dl = c.delta;
        iter = 1;
        stamp(4, __builtin_amdgcn_s_memtime());
        while (phase != PH_DONE) {
            if constexpr (DIAG) {   // time per phase: the previous pass of this loop went to its phase's bucket
                const long long now = __builtin_amdgcn_s_memtime();
                if (ph_prev == PH_POLISH) cyc_pol += now - t_prev;
                t_prev = now;
                ph_prev = phase;
            }
            // ---- K = P + ks I + A' diag(kb, kr) A (row r, half h from the scratch), then the sweep: K <- -K^-1 ----
            const double kb = (phase == PH_ADMM) ? rb : (actb ? 1.0 / dl : 0.0);
            const double kr = (phase == PH_ADMM) ? rr : (actr ? 1.0 / dl : 0.0);
            const double ks = (phase == PH_ADMM) ? sig : dl;
            {
                const double kr_up = exch(kr, +2);
                const double a_rp = exch(a_rm, +2);   // Er(r+2) D(r)
                const double dii = ks + kb * a_b * a_b + kr * a_r * a_r + kr_up * a_rp * a_rp;
                const double dp = -kr_up * a_r_up * a_rp;          // (r, r+2)
                const double dm = -kr * a_r * a_rm;                // (r, r-2): row r-2's dp, the same product
                // The band goes into P in the scratch (row r's half-0 lane adds its diagonal and its (r, r +- 2) entries),
                // both lanes load the row half as it stands -- no per-entry selects (their masks, invariant across the
                // solve, are what the compiler would hoist and spill) -- and the three entries are restored.
                double* const prow = Prow(r);
                double o_dg = 0.0, o_sp = 0.0, o_sm = 0.0;
                const bool has_sp = own && r + 2 < n, has_sm = own && has_prev;
                if (SPLIT_GHOST && phase == PH_ADMM && h == 0) {   // this row's constants for the ghost update
                    double* g = s_gh[r];
                    g[0] = a_r; g[1] = a_rm; g[2] = slr; g[3] = sur; g[4] = rr; g[5] = 1.0 / rr;
                }
                if (own && h == 0) {
                    o_dg = prow[r];
                    prow[r] = o_dg + dii;
                    if (has_sp) { o_sp = prow[r + 2]; prow[r + 2] = o_sp + dp; }
                    if (has_sm) { o_sm = prow[r - 2]; prow[r - 2] = o_sm + dm; }
                }
                __syncthreads();
                const double2* p2 = reinterpret_cast<const double2*>(prow + h * H);
#pragma unroll
                for (int i = 0; i < H; i += 2) {
                    const double2 pv = p2[i / 2];
                    Kh[i] = pv.x;
                    Kh[i + 1] = pv.y;
                }
                __syncthreads();
                if (own && h == 0) {
                    prow[r] = o_dg;
                    if (has_sp) prow[r + 2] = o_sp;
                    if (has_sm) prow[r - 2] = o_sm;
                }
            }
            // The sweep: pivot p in half hp = p / H, q = p mod H.  Before pivot p both halves are rotated by q: register
            // i of half h holds column h H + (i + q) mod H, so column p is register 0 of half hp.  The pivot column
            // (= the pivot row, K symmetric) is published as two contiguous rotated slices per half, so each lane reads
            // its rotated pivot-row entries from one 16-byte aligned slice.  Pivots past n (padding) only rotate.
            bool ok = true;
            [[maybe_unused]] const long long t_sw = DIAG ? (long long)__builtin_amdgcn_s_memtime() : 0;
            // SPLIT_BLOCK2: pivots p, p + 1 (q even, both in half hp: H and n are even) as one 2 x 2 block -- the
            // composition of the two single sweeps, with the second pivot's d and every coefficient formed as the
            // sequential sweep forms them (a = K_pp, b = K_p+1,p, c = K_p+1,p+1; 1/a; d2 = c - (b/a) b; 1/d2):
            //   row r outside the block: u = K_rp, v = K_r,p+1; beta = (v - (u/a) b)/d2, alpha = (u - beta b)/a;
            //     K_rj <- K_rj - alpha K_pj - beta K_p+1,j, and (K_rp, K_r,p+1) <- (alpha, beta);
            //   rows p, p + 1: the rows of the block inverse G (g00 = 1/a + (b/a)^2/d2, g01 = g10 = -(b/a)/d2,
            //     g11 = 1/d2) times the pivot rows, from an exact zero row, and (K_pp .. ) <- -G.
            // The two pivot columns are published as two slices (A: column p, B: column p + 1) in the rotated layout
            // of the single sweep; registers rotate by two per block.  The same algebra as two single pivots, one
            // barrier and one LDS round instead of two; the rounding of the composed coefficients differs in the
            // last bits from the sequential form.
            if constexpr (SPLIT_BLOCK2) {
                for (int hp = 0; hp < 2; ++hp) {
#pragma unroll 2
                    for (int q = 0; q < H; q += 2) {
                        const int pv = hp * H + q;
                        if (pv >= n) {   // a padding pair: identity rows, a rotation by two only
                            const double k0 = Kh[0], k1 = Kh[1];
#pragma unroll
                            for (int i = 2; i < H; ++i) Kh[i - 2] = Kh[i];
                            Kh[H - 2] = k0;
                            Kh[H - 1] = k1;
                            continue;
                        }
                        double e0, e1, f0, f1;
                        swap32(Kh[0], e0, e1);
                        swap32(Kh[1], f0, f1);
                        const double u = hp ? e1 : e0;   // K[r][p]
                        const double v = hp ? f1 : f0;   // K[r][p + 1]
                        const int par = (pv >> 1) & 1;
                        double* const slA = &s_pv2[par][0][0][0];
                        double* const slB = &s_pv2[par][1][0][0];
                        if (r < NR) {
                            slA[(r / H) * SPV + (r % H) + h * H] = u;
                            slB[(r / H) * SPV + (r % H) + h * H] = v;
                        }
                        [[maybe_unused]] long long ts0 = 0;
                        if constexpr (DIAG) ts0 = __builtin_amdgcn_s_memtime();
                        __syncthreads();
                        if constexpr (DIAG) cyc_swb += (long long)__builtin_amdgcn_s_memtime() - ts0;
                        const double2 ab = *reinterpret_cast<const double2*>(&slA[hp * SPV + q]);   // K_pp, K_p+1,p
                        const double cc = slB[hp * SPV + q + 1];                                     // K_p+1,p+1
                        // the pivot rows' entries of this half, rotated: K[p | p + 1][h H + (i + q) mod H]
                        const double2* pa2 =
                            reinterpret_cast<const double2*>(__builtin_assume_aligned(slA + h * SPV + q, 16));
                        const double2* pb2 =
                            reinterpret_cast<const double2*>(__builtin_assume_aligned(slB + h * SPV + q, 16));
                        double2 ca[2], cb[2];
#pragma unroll
                        for (int i = 0; i < 2; ++i) {
                            ca[i] = pa2[i];
                            cb[i] = pb2[i];
                        }
                        const double a = ab.x, bb = ab.y;
                        const double ainv = rcp_nr(a);
                        const double t = bb * ainv;
                        const double d2 = fma(-t, bb, cc);
                        ok = ok && (a > 0.0) && (d2 > 0.0);
                        const double d2inv = rcp_nr(d2);
                        const bool p0 = (r == pv), p1 = (r == pv + 1);
                        const double td = t * d2inv;
                        const double beta = fma(-(u * ainv), bb, v) * d2inv;
                        const double alpha = fma(-beta, bb, u) * ainv;
                        // coefficients of the two pivot rows: -(alpha, beta) outside the block, G's row inside
                        const double cA = p0 ? fma(td, t, ainv) : (p1 ? -td : -alpha);
                        const double cB = p0 ? -td : (p1 ? d2inv : -beta);
                        if ((p0 || p1) && !TGMPC_SPLIT_NOZERO_TIMING) {
#pragma unroll
                            for (int i = 0; i < H; ++i) Kh[i] = 0.0;
                        }
                        [[maybe_unused]] long long ts2 = 0;
                        if constexpr (DIAG) {
                            ts2 = __builtin_amdgcn_s_memtime();
                            cyc_sw1 += ts2 - ts0;
                        }
                        // old registers 0, 1 (the pivot columns in half hp, ordinary columns in the other half)
                        const double w0 = fma3(cA, ca[0].x, fma(cB, cb[0].x, Kh[0]));
                        const double w1 = fma3(cA, ca[0].y, fma(cB, cb[0].y, Kh[1]));
                        Kh[0] = fma3(cA, ca[1].x, fma(cB, cb[1].x, Kh[2]));
                        Kh[1] = fma3(cA, ca[1].y, fma(cB, cb[1].y, Kh[3]));
#pragma unroll
                        for (int c4 = 4; c4 < H; c4 += 4) {   // columns c4 .. c4 + 3 (double2 c4 / 2, c4 / 2 + 1)
#pragma unroll
                            for (int i = 0; i < 2; ++i) {
                                ca[i] = pa2[c4 / 2 + i];
                                cb[i] = pb2[c4 / 2 + i];
                            }
#pragma unroll
                            for (int i = 0; i < 2; ++i) {
                                const int j = c4 + 2 * i;
                                Kh[j - 2] = fma3(cA, ca[i].x, fma(cB, cb[i].x, Kh[j]));
                                Kh[j - 1] = fma3(cA, ca[i].y, fma(cB, cb[i].y, Kh[j + 1]));
                            }
                        }
                        Kh[H - 2] = (h == hp) ? -cA : w0;
                        Kh[H - 1] = (h == hp) ? -cB : w1;
                        if constexpr (DIAG) cyc_sw2 += (long long)__builtin_amdgcn_s_memtime() - ts2;
                    }
                }
            } else
            for (int hp = 0; hp < 2; ++hp) {
#pragma unroll 2
                for (int q = 0; q < H; ++q) {
                    const int pv = hp * H + q;
                    if (pv >= n) {   // padding pivot: the identity row, a rotation only
                        const double k0 = Kh[0];
#pragma unroll
                        for (int i = 1; i < H; ++i) Kh[i - 1] = Kh[i];
                        Kh[H - 1] = k0;
                        continue;
                    }
                    double e0, e1;
                    swap32(Kh[0], e0, e1);
                    const double kp = hp ? e1 : e0;            // K[r][p]: register 0 of the half holding column p
                    const int par = pv & 1, off = q & 1;
                    double* const sl = &s_pv[par][0][0];
                    // row r publishes its K[r][p] = K[p][r] at slice position (r mod H) and (r mod H) + H of half r / H
                    if (r < NR) sl[(r / H) * SPV + off + (r % H) + h * H] = kp;
                    [[maybe_unused]] long long ts0 = 0;
                    if constexpr (DIAG) ts0 = __builtin_amdgcn_s_memtime();
                    __syncthreads();
                    if constexpr (DIAG) cyc_swb += (long long)__builtin_amdgcn_s_memtime() - ts0;
                    const double d = sl[hp * SPV + off + q];
                    // rotated pivot-row entries of this half: K[p][h H + (i + q) mod H] at sl[h SPV + off + q + i] --
                    // the first chunk read with d, ahead of the reciprocal and the pivot row's branch
                    const double2* pr2 =
                        reinterpret_cast<const double2*>(__builtin_assume_aligned(sl + h * SPV + off + q, 16));
                    double2 cur[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) cur[i] = pr2[i];
                    ok = ok && (d > 0.0);
                    const double dinv = rcp_nr(d);
                    const bool piv = (r == pv);
                    const double fd = kp * dinv;
                    const double be = piv ? dinv : -fd;
                    const double k0 = piv ? -dinv : fd;
                    if (piv && !TGMPC_SPLIT_NOZERO_TIMING) {   // the pivot row becomes K_pj / d: an exact zero row plus be * K_pj
#pragma unroll
                        for (int i = 0; i < H; ++i) Kh[i] = 0.0;
                    }
                    [[maybe_unused]] long long ts2 = 0;
                    if constexpr (DIAG) {
                        ts2 = __builtin_amdgcn_s_memtime();
                        cyc_sw1 += ts2 - ts0;
                    }
                    const double last = fma3(be, cur[0].x, Kh[0]);   // column h H + q (the non-pivot half's entry)
#pragma unroll
                    for (int i0 = 0; i0 < H; i0 += 8) {
                        double2 nxt[4];
                        if (i0 + 8 < H) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) nxt[i] = pr2[(i0 + 8) / 2 + i];
                        }
#pragma unroll
                        for (int i = 0; i < 4; ++i) {
                            const int j = i0 + 2 * i;
                            // (three-address fma: the rotated destination is written directly, no register copies)
                            if (j > 0) Kh[j - 1] = fma3(be, cur[i].x, Kh[j]);
                            Kh[j] = fma3(be, cur[i].y, Kh[j + 1]);
                        }
                        if (i0 + 8 < H) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) cur[i] = nxt[i];
                        }
                    }
                    Kh[H - 1] = (h == hp) ? k0 : last;
                    if constexpr (DIAG) cyc_sw2 += (long long)__builtin_amdgcn_s_memtime() - ts2;
                }
            }
#pragma unroll
            for (int i = 0; i < H; ++i) Kh[i] = -Kh[i];
            __syncthreads();
            if constexpr (DIAG) {
                cyc_sweep += (long long)__builtin_amdgcn_s_memtime() - t_sw;
                ++n_fact;
            }
            if (!ok) {
                if (phase == PH_ADMM) { status = TRAJ_STATUS_SOLVER_ERROR; break; }
                if (c.polish_mode == 1 && rounds < c.polish_max_rounds && iter < c.max_iter) {
                    ++rounds;
                    escale *= 1e-2;
                    ++iter;
                    phase = PH_ADMM;
                } else {
                    phase = PH_DONE;
                }
                continue;
            }
            if (phase == PH_ADMM) {
                bool converged = false, refactor = false;
                int chk = c.check_interval - (iter - 1) % c.check_interval;
                const double oma = 1.0 - alpha;
                const double rib = 1.0 / rb, rir = 1.0 / rr;
                // SPLIT_GHOST: row r also runs row r + 2's rate-row update (zr, yr: the same operations on the same
                // values, so the same bits), which is all that A' w needs of row r + 2 -- so the iteration exchanges
                // only xt (both neighbours in one round) and has two barriers (the broadcast, the exchange), not three.
                const double2* const gq = reinterpret_cast<const double2*>(s_gh[r + 2]);
                const bool has_up = own && r + 2 < n;
                for (; iter <= c.max_iter; ++iter) {
                    const double wb = fma(rb, zb, -yb), wr = fma(rr, zr, -yr);
                    double rp_up;
                    double2 g01, g23, g45;
                    if constexpr (SPLIT_GHOST) {
                        g01 = gq[0]; g23 = gq[1]; g45 = gq[2];   // a_r, a_rm | slr, sur | rr, 1 / rr of row r + 2
                        rp_up = has_up ? g01.y * fma(g45.x, zr_g, -yr_g) : 0.0;
                    } else {
                        rp_up = exch(a_rm * wr, +2);
                    }
                    const double atw = fma(a_b, wb, fma(a_r, wr, -rp_up));
                    const double xt = Kmul(fma(sig, x, atw - qi));
                    double xt_dn;
                    if constexpr (SPLIT_GHOST) {
                        double* buf = s_ex[xb & 3];
                        xb++;
                        if (h == 0) buf[r] = xt;
                        __syncthreads();
                        xt_dn = (own && r >= 2) ? buf[r - 2] : 0.0;
                        const double xt_up = has_up ? buf[r + 2] : 0.0;
                        // row r + 2's update (its xt_dn is this row's xt)
                        const double ztr_g = fma(g01.x, xt_up, -(g01.y * xt));
                        const double zrr_g = fma(alpha, ztr_g, oma * zr_g);
                        const double nzr_g = clamp_mm(fma(g45.y, yr_g, zrr_g), g23.x, g23.y);
                        yr_g = fma(g45.x, zrr_g - nzr_g, yr_g);
                        zr_g = nzr_g;
                    } else {
                        xt_dn = exch(xt, -2);
                    }
                    const double ztb = a_b * xt, ztr = fma(a_r, xt, -(a_rm * xt_dn));
                    const double xn = fma(alpha, xt, oma * x);
                    const double zrb = fma(alpha, ztb, oma * zb), zrr = fma(alpha, ztr, oma * zr);
                    const double nzb = clamp_mm(fma(rib, yb, zrb), slb, sub), nzr = clamp_mm(fma(rir, yr, zrr), slr, sur);
                    yb = fma(rb, zrb - nzb, yb);
                    yr = fma(rr, zrr - nzr, yr);
                    x = xn;
                    zb = nzb;
                    zr = nzr;
                    if (--chk == 0) {
                        chk = c.check_interval;
                        rs0 = residuals(x, zb, zr, yb, yr);
                        if (rs0.pr <= escale * rs0.eps_p && rs0.dr <= escale * rs0.eps_d) { converged = true; break; }
                        if (c.adaptive_rho) {
                            double est = rho * sqrt((rs0.prs / (rs0.pn + DIV_TOL)) / (rs0.drs / (rs0.dn + DIV_TOL) + DIV_TOL));
                            est = fmin(fmax(est, RHO_MIN), RHO_MAX);
                            if (est > rho * c.adaptive_rho_tol || est < rho / c.adaptive_rho_tol) {
                                rho = est;
                                rb = rho_for(slb, sub, rho);
                                rr = rho_for(slr, sur, rho);
                                refactor = true;
                                ++iter;
                                break;
                            }
                        }
                    }
                }
                if (refactor && iter <= c.max_iter) continue;
                if (converged) status = TRAJ_STATUS_OPTIMAL;
                else {
                    iter = c.max_iter;
                    rs0 = residuals(x, zb, zr, yb, yr);
                    status = (rounds > 0 && rs0.pr <= rs0.eps_p && rs0.dr <= rs0.eps_d) ? TRAJ_STATUS_OPTIMAL
                             : (rs0.pr <= 10.0 * rs0.eps_p && rs0.dr <= 10.0 * rs0.eps_d) ? TRAJ_STATUS_OPTIMAL_INACCURATE
                                                                                       : TRAJ_STATUS_USER_LIMIT;
                }
                if (status == TRAJ_STATUS_OPTIMAL && c.polish) {
                    // OSQP active sets: lower if z - l < -y, upper if u - z < y
                    actb = own ? ((zb - slb < -yb) ? -1 : ((sub - zb < yb) ? 1 : 0)) : 0;
                    actr = own ? ((zr - slr < -yr) ? -1 : ((sur - zr < yr) ? 1 : 0)) : 0;
                    ps = 1;
                    phase = PH_POLISH;
                } else {
                    phase = PH_DONE;
                }
                continue;
            }
            // ---- polish: K^-1 = M^-1, M = P + delta I + Ar' Ar / delta (the eliminated reduced KKT) ----
            {
                const double bbv = actb < 0 ? slb : (actb > 0 ? sub : 0.0);
                const double brv = actr < 0 ? slr : (actr > 0 ? sur : 0.0);
                double px_ = 0.0, pyb = 0.0, pyr = 0.0;
                double r1 = -qi, r2b = actb ? bbv : 0.0, r2r = actr ? brv : 0.0;
                double axb = 0.0, axr = 0.0;
                for (int rf = 0; rf <= c.polish_refine_iter; ++rf) {
                    const double tv = Kmul(r1 + ATw(actb ? r2b / dl : 0.0, actr ? r2r / dl : 0.0));
                    double tb, tr;
                    Ax(tv, tb, tr);
                    px_ += tv;
                    if (actb) pyb += (tb - r2b) / dl;
                    if (actr) pyr += (tr - r2r) / dl;
                    if (rf == c.polish_refine_iter) break;
                    const double Pxv = Pmul(px_);
                    const double atyv = ATw(pyb, pyr);
                    r1 = -qi - Pxv - atyv;
                    Ax(px_, axb, axr);
                    r2b = actb ? bbv - axb : 0.0;
                    r2r = actr ? brv - axr : 0.0;
                }
                Ax(px_, axb, axr);
                if (c.polish_mode == 0) {
                    // z = proj(Ax + y), y = Ax + y - z (OSQP project_normalcone); accept if the residuals drop
                    const double ztb = axb + pyb, ztr = axr + pyr;
                    const double nzb = clampd(ztb, slb, sub), nzr = clampd(ztr, slr, sur);
                    const double nyb = ztb - nzb, nyr = ztr - nzr;
                    const Res rp = residuals(px_, nzb, nzr, nyb, nyr);
                    const bool okp = (rp.pr < rs0.pr && rp.dr < rs0.dr) || (rp.pr < rs0.pr && rs0.dr < 1e-10) ||
                                     (rp.dr < rs0.dr && rs0.pr < 1e-10);
                    if (okp) {
                        x = px_; zb = nzb; zr = nzr; yb = nyb; yr = nyr;
                        pol = 1;
                    }
                    phase = PH_DONE;
                    continue;
                }
                // exact mode: the KKT certificate in the unscaled problem
                const double Pxv = Pmul(px_);
                const double atyv = ATw(pyb, pyr);
                const double tol = c.cert_tol;
                double v[2];
                double lb_ = ch ? c.u_lo[1] : c.u_lo[0], ub_ = ch ? c.u_hi[1] : c.u_hi[0];
                double lr_ = ch ? c.du_lo[1] : c.du_lo[0], ur_ = ch ? c.du_hi[1] : c.du_hi[0];
                if (kk == 0) { lr_ += up[ch]; ur_ += up[ch]; }
                v[0] = own ? fabs(Dinv * (Pxv + qi + atyv)) * csinv : 0.0;            // stationarity
                v[1] = own ? fmax(fabs(Dinv * qi), fabs(Dinv * Pxv)) * csinv : 0.0;  // gradient scale
                block_max(v);
                const double gsc = fmax(1.0, v[1]);
                int okc = v[0] <= tol * gsc;
                if (own) {
                    const double axu = axb * Ebinv, arv = axr * Erinv;
                    if (slb > -INFTY && axu < lb_ - tol * (1.0 + fabs(lb_))) okc = 0;
                    if (sub < INFTY && axu > ub_ + tol * (1.0 + fabs(ub_))) okc = 0;
                    if (slr > -INFTY && arv < lr_ - tol * (1.0 + fabs(lr_))) okc = 0;
                    if (sur < INFTY && arv > ur_ + tol * (1.0 + fabs(ur_))) okc = 0;
                    const double ybu = pyb * Eb * csinv, yru = pyr * Er * csinv;
                    if (actb < 0 && ybu > tol * gsc) okc = 0;
                    if (actb > 0 && ybu < -tol * gsc) okc = 0;
                    if (actr < 0 && yru > tol * gsc) okc = 0;
                    if (actr > 0 && yru < -tol * gsc) okc = 0;
                }
                double fo[1] = {okc ? 0.0 : 1.0};
                block_max(fo);
                if (fo[0] == 0.0) {
                    x = px_;
                    zb = clampd(axb, slb, sub);
                    zr = clampd(axr, slr, sur);
                    yb = pyb;
                    yr = pyr;
                    pol = ps + 16 * rounds;
                    phase = PH_DONE;
                    continue;
                }
                if (ps < c.polish_max_pass) {
                    // primal-dual active-set update with the OSQP rule on the polished (Ax, y)
                    actb = own ? ((axb - slb < -pyb) ? -1 : ((sub - axb < pyb) ? 1 : 0)) : 0;
                    actr = own ? ((axr - slr < -pyr) ? -1 : ((sur - axr < pyr) ? 1 : 0)) : 0;
                    ++ps;
                    continue;
                }
                if (rounds < c.polish_max_rounds && iter < c.max_iter) {
                    // not certified: continue ADMM to a 100x tighter tolerance, then polish again
                    ++rounds;
                    escale *= 1e-2;
                    ++iter;
                    phase = PH_ADMM;
                    continue;
                }
                phase = PH_DONE;
            }
        }
        if constexpr (DIAG) {
            const long long now = __builtin_amdgcn_s_memtime();
            if (ph_prev == PH_POLISH) cyc_pol += now - t_prev;
            stamp(6, now);
            stamp(5, cyc_sweep);
            stamp(8, n_fact);
            stamp(10, cyc_pol);
            stamp(15, cyc_swb);
            stamp(16, cyc_xb);
            stamp(17, cyc_sw1);
            stamp(18, cyc_sw2);
        }
        if (iter > c.max_iter) iter = c.max_iter;
        xsol = D * x;
        if (CLOSED && a.wsWarm && t == 0) {
            double* wv = a.wsWarm + 4 * (size_t)b;
            const double w[3] = {rho, (status == TRAJ_STATUS_OPTIMAL || status == TRAJ_STATUS_OPTIMAL_INACCURATE) ? 1.0 : 0.0,
                                 (double)iter};
            for (int i = 0; i < 3; ++i) {
                if (FUSED) st_coh(wv + i, w[i]);
                else wv[i] = w[i];
            }
        }
    } else {
        status = early;
        iter = 0;
        if (CLOSED && a.wsWarm && t == 0) {
            if (FUSED) {
                st_coh(a.wsWarm + 4 * (size_t)b + 1, 0.0);
                st_coh(a.wsWarm + 4 * (size_t)b + 2, 0.0);
            } else {
                a.wsWarm[4 * (size_t)b + 1] = 0.0;
                a.wsWarm[4 * (size_t)b + 2] = 0.0;
            }
        }
    }

    // ---- outputs (:257-275): U, X_opt by the linear model, the objective, u_cmd (CLOSED: the plant update) ----
    const bool good = (status == TRAJ_STATUS_OPTIMAL || status == TRAJ_STATUS_OPTIMAL_INACCURATE);
    const double nan = __builtin_nan("");
    double* const Ub = s_bc[0];
    __syncthreads();
    if (h == 0) Ub[r] = own ? xsol : 0.0;
    __syncthreads();
    if constexpr (CLOSED) {
        // plant x <- x + Ts f(x, u_cmd) (main.py:97), u_prev <- u_cmd (:101); the history and this step's outcome
        if (t == 0) {
            const double uc0 = good ? Ub[0] : up[0], uc1 = good ? Ub[1] : up[1];
            double xs[6], f[6], u[2] = {uc0, uc1};
            for (int i = 0; i < 6; ++i) xs[i] = x0[i];
            f_cont(p, xs, u, f);
            for (int i = 0; i < 6; ++i) {
                const double xn = xs[i] + c.Ts * f[i];
                if (FUSED) st_coh(a.x_state + 6 * (size_t)b + i, xn);
                else a.x_state[6 * (size_t)b + i] = xn;
                if (a.hist_x) a.hist_x[((size_t)b * (a.hist_T + 1) + tstep + 1) * 6 + i] = xn;
            }
            if (FUSED) {
                st_coh(a.u_state + 2 * (size_t)b, uc0);
                st_coh(a.u_state + 2 * (size_t)b + 1, uc1);
            } else {
                a.u_state[2 * (size_t)b] = uc0;
                a.u_state[2 * (size_t)b + 1] = uc1;
            }
            if (a.hist_u) {
                a.hist_u[((size_t)b * a.hist_T + tstep) * 2] = uc0;
                a.hist_u[((size_t)b * a.hist_T + tstep) * 2 + 1] = uc1;
            }
            if (a.status) a.status[(size_t)step * a.B + b] = status;
            if (a.iters) a.iters[(size_t)step * a.B + b] = iter;
            if (FUSED) {
                // mean iterations per step of this launch (the next launch's order), accumulated
                if (a.wsWarm) {
                    double* m = a.wsWarm + 4 * (size_t)b + 3;
                    const double acc = (step == 0 ? 0.0 : ld_coh(m)) + iter;
                    st_coh(m, (step == a.nsteps - 1) ? acc / a.nsteps : acc);
                }
                // hand the instance to whichever workgroup takes its next step: the sc1 state stores complete
                // (vmcnt(0)), then the step counter is stored sc1
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&a.queue[2 + b], step + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        stamp(9, iter);
        stamp(7, __builtin_amdgcn_s_memtime());
        __syncthreads();
        continue;
    }
    // X_{k+1} = A_k X_k + B_k U_k + g_k, stage by stage (thread i < 6: state i)
    double* const Xs = s_xs;
    if (t < 6) Xs[t] = x0[t];
    __syncthreads();
    for (int k = 0; k < N; ++k) {
        if (t < 6) {
            double v = 0.0;
            for (int cc = 0; cc < 6; ++cc) v += gA[RA * k + t * 6 + cc] * Xs[6 * k + cc];
            v += gB[RB * k + t * 2] * Ub[2 * k] + gB[RB * k + t * 2 + 1] * Ub[2 * k + 1] + gg[RG * k + t];
            Xs[6 * (k + 1) + t] = v;
        }
        __syncthreads();
    }
    // objective: the cost of :217-250 at (X_opt, U_opt), k = t over the threads, summed in a fixed order
    double op = 0.0;
    for (int k = t; k <= N; k += NT) {
        const double* X = Xs + 6 * k;
        const double s = s_sc[k][0], co = s_sc[k][1];
        const double ec = s * (X[0] - pref[3 * k]) - co * (X[1] - pref[3 * k + 1]);
        const double ep = X[2] - pref[3 * k + 2];
        const double ev = X[3] - s_vr[k];
        op += c.q_c * ec * ec + c.q_phi * ep * ep + c.q_vx * ev * ev;
        if (k < N) {
            const double u0 = Ub[2 * k], u1 = Ub[2 * k + 1];
            const double d0 = u0 - (k == 0 ? up[0] : Ub[2 * k - 2]);
            const double d1 = u1 - (k == 0 ? up[1] : Ub[2 * k - 1]);
            op += u0 * (c.R[0] * u0 + c.R[1] * u1) + u1 * (c.R[2] * u0 + c.R[3] * u1);
            op += d0 * (c.Rd[0] * d0 + c.Rd[1] * d1) + d1 * (c.Rd[2] * d0 + c.Rd[3] * d1);
        }
    }
    // (every thread's partial -- not only half 0's rows: block_sum takes half-0 lanes, so sum by thread here)
    op = wave_sum_dpp(op);
    if (lane == 0) s_red[wid * 8] = op;
    __syncthreads();
    double obj = 0.0;
    for (int w = 0; w < WAVES; ++w) obj += s_red[w * 8];
    if (t == 0) {
        a.u_cmd[2 * b] = good ? Ub[0] : up[0];
        a.u_cmd[2 * b + 1] = good ? Ub[1] : up[1];
        a.status[b] = status;
        if (a.objective) a.objective[b] = good ? obj : nan;
        if (a.iters) a.iters[b] = iter;
        if (a.polished) a.polished[b] = pol;
    }
    if (a.U_opt && own && h == 0) a.U_opt[(size_t)b * 2 * N + ch * N + kk] = good ? xsol : nan;
    if (a.X_opt)
        for (int i = t; i < 6 * (N + 1); i += NT) {
            const int rr = i / (N + 1), k = i % (N + 1);
            a.X_opt[(size_t)b * 6 * (N + 1) + i] = good ? Xs[6 * k + rr] : nan;
        }
    }   // work items
}

}  // namespace tgmpc
