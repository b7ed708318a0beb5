// mpc_common.h -- shared definitions of the batched MPC step kernels for gfx950 (mpc_linearize.h,
// mpc_solve.h).
//
// Reference hot path: MPC/mpc_6stati.py:120-275 (mpc_step).  Per instance the kernel runs
//   1. nominal rollout          :165-172  x_{k+1} = x_k + Ts f(x_k, u_prev)
//   2. linearize/discretize     :175-178  central differences (:73-97), A = I + Ts Jx, B = Ts Ju,
//                                          g = x + Ts f - A x - B u (:99-109)
//   3. the TV-LQ QP             :180-250  condensed over U (X eliminated by the dynamics)
//   4. the solve                :252-262  OSQP's ADMM (Ruiz scaling, sigma/alpha, adaptive rho,
//                                          OSQP termination) + polish, as restated in oracle/
//   5. status / info            :257-275  u_cmd = U[:,0] or u_prev; X_opt by the linear model
//
// Layout (DESIGN.md "Kernel"): thread i (< n = 2N) owns QP variable i = 2k + channel, its box row
// and its rate row.  Matrices live ROW-PER-LANE in registers: the KKT matrix
// K = P + sigma I + A' diag(rho) A is inverted in place by the symmetric sweep operator
// (n pivots, each a broadcast of one column through LDS), so every ADMM iteration is one dense
// register mat-vec (n FMAs/lane) plus two +-2 neighbour exchanges for the banded constraint rows.
// The scaled cost matrix P (needed for residuals, rho updates and polish) stays in LDS.
// Everything is float64, like the reference.
#pragma once
#include "physics.h"

#ifndef TGMPC_DPP_BC
#define TGMPC_DPP_BC 0   // DPP moves with bound_ctrl (see dpp_d; the Makefile turns it on for mpc_inst.hip)
#endif

namespace tgmpc {

constexpr double INFTY = 1e30;
constexpr double DIV_TOL = 1e-30;
constexpr double MIN_SCALING = 1e-4;
constexpr double MAX_SCALING = 1e4;
constexpr double RHO_MIN = 1e-6;
constexpr double RHO_MAX = 1e6;
constexpr double RHO_TOL = 1e-4;
constexpr double RHO_EQ_OVER_INEQ = 1e3;

struct PathArgs {
    int kmax;
    const int* kind;
    const double* pc;
    const int* nk;
    const double* xk;
    const double* coef;
};

// fused closed loop: instances per workgroup at most (the grid is the resident workgroups, or more)
#define TRAJ_FUSED_MAX_PER_WG 8

struct KArgs {
    traj_vehicle_params p;
    traj_mpc_config c;
    int B;
    const double* x0;        // [B,6]  (closed loop: state, updated in place)
    const double* u_prev;    // [B,2]
    const double* path_ref;  // [B,N+1,3] (unused in closed loop)
    const double* vref;      // [B,N+1]
    const double* Ad;        // [B,N,6,6] (QP-only mode)
    const double* Bd;
    const double* gd;
    double* u_cmd;           // [B,2]
    int* status;
    double* objective;
    double* X_opt;           // [B,6,N+1]
    double* U_opt;           // [B,2,N]
    int* iters;
    int* polished;
    // closed loop
    PathArgs path;
    double* x_state;         // [B,6]
    double* u_state;         // [B,2]
    int t, hist_T;
    double* hist_x;          // [B,T+1,6]
    double* hist_u;          // [B,T,2]
    long long* dbg;          // diagnostics: per-block phase stamps (s_memtime) + counters, or null
    double* wsA;             // linearization outputs (workspace): [B,N,6,6], [B,N,6,2], [B,N,6]
    double* wsB;
    double* wsg;
    double* wsXF;            // rollout record (x_k, f_k) per stage: [B,N,12]
    double* wsWarm;          // closed loop: per instance [rho, valid, ADMM iterations, 0] of the previous step
    const int* perm;         // closed loop: instance order (longest previous solve first), or null
    int nsteps;              // > 0: fused closed loop, nsteps steps per launch (status / iters [nsteps, B])
    int fused_grid;          // fused: workgroups to launch (0: the resident slots; traj_debug_fused_grid)
    int* queue;              // fused: [0] next work item, [1] error flag, [2 + b] completed steps of b,
                             //        [2 + B + b] steps of b claimed (drawn from the queue or run ahead)
    int spin_limit;          // fused: polls of a step counter before a hand-off is declared lost
    long long* dbg_items;    // fused diagnostics: per work item q [4]: drawn, wait over, done (100 MHz), slot
    int lead_steps, lead_h;  // fused: the heaviest lead_h ranks run lead_steps steps ahead in the queue order
    int run_ahead;           // fused: a workgroup keeps its instance for the next step while that step is at most
                             //        run_ahead levels past the queue's draw front (0: every step from the queue)
    int wps;                 // fused: waves per SIMD of the kernel instance to launch (2, or 3 where built)
};

// Fused closed loop: coherent (sc1) stores and loads of an instance's state handed between workgroups on any XCD
// (mpc_solve.h explains the protocol)
__device__ __forceinline__ void st_coh(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_coh(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double limit_scaling(double v) {
    return v < MIN_SCALING ? 1.0 : (v > MAX_SCALING ? MAX_SCALING : v);
}

// reference path y(x), dy/dx for the closed-loop window (DESIGN.md "reference paths")
__device__ inline void path_eval(const PathArgs& pa, int b, double x, double& y, double& dy) {
    int kind = pa.kind[b];
    const double* c = pa.pc + 4 * b;
    if (kind == 0) {
        y = c[0] + x * (c[1] + x * (c[2] + x * c[3]));
        dy = c[1] + x * (2.0 * c[2] + x * 3.0 * c[3]);
    } else if (kind == 1) {
        double a = c[1] * x + c[2];
        double s, co;
        pm_sincos(a, &s, &co);
        y = c[0] * s + c[3];
        dy = c[0] * c[1] * co;
    } else {
        int nk = pa.nk[b];
        const double* xk = pa.xk + (size_t)pa.kmax * b;
        const double* cf = pa.coef + (size_t)(pa.kmax - 1) * 4 * b;
        if (x <= xk[0]) {
            y = cf[0] + cf[1] * (x - xk[0]);
            dy = cf[1];
        } else if (x >= xk[nk - 1]) {
            const double* q = cf + 4 * (nk - 2);
            double h = xk[nk - 1] - xk[nk - 2];
            double ye = q[0] + h * (q[1] + h * (q[2] + h * q[3]));
            double se = q[1] + h * (2.0 * q[2] + h * 3.0 * q[3]);
            y = ye + se * (x - xk[nk - 1]);
            dy = se;
        } else {
            int j = 0;
            while (j < nk - 2 && x >= xk[j + 1]) ++j;
            const double* q = cf + 4 * j;
            double tt = x - xk[j];
            y = q[0] + tt * (q[1] + tt * (q[2] + tt * q[3]));
            dy = q[1] + tt * (2.0 * q[2] + tt * 3.0 * q[3]);
        }
    }
}

template <int V>
__device__ __forceinline__ void wave_max(double (&v)[V]) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
            double o = __shfl_xor(v[i], off, 64);
            v[i] = (o > v[i] || o != o) ? o : v[i];
        }
    }
}

// a wave-uniform double moved to SGPRs (readfirstlane), so the compiler stops carrying it in VGPRs
__device__ __forceinline__ double uniformize(double v) {
    const long long bits = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(bits & 0xffffffffLL));
    const int hi = __builtin_amdgcn_readfirstlane((int)(bits >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// 1/d for a normal, finite d: v_rcp_f64 + two Newton steps (the IEEE division sequence without its
// scale / fix-up steps; within an ulp of 1.0 / d)
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(fma(-d, r, 1.0), r, r);
    r = fma(fma(-d, r, 1.0), r, r);
    return r;
}

// max(a, b) and max(a, |b|) as ONE v_max_f64.  In the default IEEE mode fmax(a, fabs(b)) compiles to a
// canonicalizing v_max_f64 of |b| with itself and then the max (two instructions per entry of a row norm); the
// operands here are arithmetic results or copies of them, never signaling NaNs, and for those the single
// instruction returns the same value (a quiet NaN operand yields the other one, as fmax does).
__device__ __forceinline__ double vmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmin(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// The ADMM projection onto [lo, hi] (lo <= hi) as v_max_f64 + v_min_f64: 2 VALU instead of two compares and four
// selects.  Equal to clampd for every non-NaN x up to the sign of a zero against a zero bound; a NaN maps to lo,
// as OSQP's own project() (c_min(c_max(z, l), u)) maps it, where clampd and the oracle pass the NaN through.  A NaN
// iterate needs NaN data (rejected before the ADMM, "Solver Error" on both sides) or an overflow inside the ADMM; the
// dual update y += rho (z~ - z) then carries the NaN on both sides, every residual is NaN, no termination test
// passes, and both end at max_iter with the same status.
__device__ __forceinline__ double clamp_mm(double x, double lo, double hi) { return vmin(vmax(x, lo), hi); }
__device__ __forceinline__ double vmax_abs(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double vmax_abs2(double a, double b) {   // max(|a|, |b|)
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// A value the compiler cannot see through (an empty asm that "modifies" it): keeps a per-lane mask from being
// folded back into a branch condition
__device__ __forceinline__ unsigned opaque_u(unsigned v) {
    asm volatile("" : "+v"(v));
    return v;
}
// m ? a : b per bit (m all ones or all zeros per lane) as two v_bfi_b32: both operands are formed on every lane
__device__ __forceinline__ double bitsel(unsigned m, double a, double b) {
    const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
    const unsigned lo = (unsigned(ua) & m) | (unsigned(ub) & ~m);
    const unsigned hi = (unsigned(ua >> 32) & m) | (unsigned(ub >> 32) & ~m);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// sqrt(x) for finite x >= 2^-767 (and NaN): the instruction sequence the compiler lowers sqrt to on gfx950 -- v_rsq_f64
// and two Newton / Goldschmidt corrections -- without its range scaling (x < 2^-767) and its +-0 / +inf class
// fix-up, so the same value in 10 instead of 17 VALU (tools/microbench/check_ops.hip compares the two on the GPU).
// The Ruiz pass's arguments are limit_scaling()'s, in [1e-4, 1e4].
__device__ __forceinline__ double sqrt_n(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    const double d0 = fma(-g, g, x);
    h = fma(h, r, h);
    g = fma(d0, h, g);
    const double d1 = fma(-g, g, x);
    return fma(d1, h, g);
}
// 1 / b where the division needs no operand scaling (b normal, |b| well inside [2^-900, 2^900]): the compiler's
// f64 division sequence without v_div_scale / v_div_fmas scaling / v_div_fixup -- the same value in 8 VALU, not 11
__device__ __forceinline__ double rcp_n(double b) {
    double y = __builtin_amdgcn_rcp(b);
    double e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    const double r = fma(-b, y, 1.0);
    return fma(r, y, y);
}

// d / c for a constant c with y = 1 / c (rounded) given: q = d y corrected once by the exact remainder
// (Markstein): r = -(q c - d) by fma, q + r y -- the IEEE quotient bit for bit for d = +-0 and every FINITE d with
// |d| >= 1e-290 whose quotient does not overflow (tools/check_cdiv.c: random operands over the whole exponent range
// for c = 2e-5, 1e-6 and every even 2..512; below 1e-290 the remainder underflows and the last bit can differ).  For
// d = +-inf, or a quotient past DBL_MAX, the remainder is inf - inf and the result NaN where IEEE gives +-inf: a
// non-finite either way, and every caller's data then fails the solver's finiteness check (status "Solver Error",
// as the oracle's +-inf does), so the statuses agree.  3 f64 operations instead of ~10.  Used for the
// central differences' (fp - fm) / (2 eps) on every path (the fused and per-step linearizations agree), the
// polish's quotients by delta and the Ruiz mean's by n.
__device__ __forceinline__ double cdiv(double d, double c, double y) {
    double q = d * y, t, r;
    asm("v_fma_f64 %0, %1, %2, -%3" : "=v"(t) : "v"(q), "v"(c), "v"(d));   // q c - d (exact)
    asm("v_fma_f64 %0, -%1, %2, %3" : "=v"(r) : "v"(t), "v"(y), "v"(q));   // q - t y
    return r;
}

// Three-address fma (v_fma_f64 dst, a, b, c): keeps the compiler from turning a register-rotating
// update into an in-place v_fmac plus register copies.
__device__ __forceinline__ double fma3(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Read NN (even) doubles from a 16-byte aligned LDS buffer as NN/2 ds_read_b128, all issued before
// the first use (the default schedule waits on each read in turn under register pressure).
template <int NN>
__device__ __forceinline__ void lds_load_all(const double* p, double (&o)[NN]) {
    const double2* p2 = reinterpret_cast<const double2*>(__builtin_assume_aligned(p, 16));
#pragma unroll
    for (int i = 0; i < NN / 2; ++i) {
        const double2 v = p2[i];
        o[2 * i] = v.x;
        o[2 * i + 1] = v.y;
    }
    __builtin_amdgcn_sched_group_barrier(0x100, NN / 2, 0);
}

// ---- DPP cross-lane moves (gfx9 data-parallel primitives: VALU, no LDS traffic) -------------
// CTRL: 0x130 wave_shl:1 (lane t receives lane t+1), 0x138 wave_shr:1 (lane t-1), 0xB1 / 0x4E
// quad_perm [1,0,3,2] / [2,3,0,1], 0x141 row_half_mirror, 0x140 row_mirror, 0x142 row_bcast:15,
// 0x143 row_bcast:31.  Lanes whose source is outside the wave, or whose row is masked off, get 0.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
#if TGMPC_DPP_BC
    if constexpr (ROW_MASK == 0xf) {
        // every row written: bound_ctrl gives the out-of-wave (or disabled) sources 0 -- the same values as an
        // old operand of 0, without the two v_mov_b32 0 that initialise it.  (Not in the 3-wave instance: there it
        // raised the scratch from 252 to 304 B/lane and cost a third of its 200-step rate.)
        lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xf, 0xf, true);
        hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xf, 0xf, true);
        return __hiloint2double(hi, lo);
    }
#endif
    lo = __builtin_amdgcn_update_dpp(0, lo, CTRL, ROW_MASK, 0xf, false);
    hi = __builtin_amdgcn_update_dpp(0, hi, CTRL, ROW_MASK, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double lane_up2(double v) { return dpp_d<0x130>(dpp_d<0x130>(v)); }  // lane t+2
__device__ __forceinline__ double lane_dn2(double v) { return dpp_d<0x138>(dpp_d<0x138>(v)); }  // lane t-2

__device__ __forceinline__ double readlane_d(double v, int l) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

// Wave-wide max of V non-negative values (NaN if any lane holds a NaN), uniform result.
// Butterfly inside rows of 16 lanes, then row_bcast 15 / 31 into lane 63, then readlane.
template <int V>
__device__ __forceinline__ void wave_max_dpp(double (&v)[V]) {
#pragma unroll
    for (int i = 0; i < V; ++i) {
        const bool nan = __ballot(v[i] != v[i]) != 0;
        double m = v[i];
        m = vmax(m, dpp_d<0xB1>(m));
        m = vmax(m, dpp_d<0x4E>(m));
        m = vmax(m, dpp_d<0x141>(m));
        m = vmax(m, dpp_d<0x140>(m));
        m = vmax(m, dpp_d<0x142, 0xa>(m));
        m = vmax(m, dpp_d<0x143, 0xc>(m));
        m = readlane_d(m, 63);
        v[i] = nan ? __builtin_nan("") : m;
    }
}

// Wave-wide sum, uniform result (same DPP pattern).
__device__ __forceinline__ double wave_sum_dpp(double v) {
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    v += dpp_d<0x142, 0xa>(v);
    v += dpp_d<0x143, 0xc>(v);
    return readlane_d(v, 63);
}


}  // namespace tgmpc
