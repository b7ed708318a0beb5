// mpc_linearize.h -- stage 1 of the MPC step: nominal rollout + central-difference linearization.
//
// Reference: MPC/mpc_6stati.py:165-178 (rollout and the N linearization points), :73-97
// (numerical_jacobian, eps = 1e-5), :99-109 (A = I + Ts Jx, B = Ts Ju, g = x + Ts f - A x - B u).
//
// Two launches, each with every lane busy:
//   rollout_kernel  one THREAD per instance runs the serial Euler rollout x_{k+1} = x_k + Ts f(x_k, u)
//                   (u = u_prev, constant) and records (x_k, f_k) per stage: [B, N, 12].
//   jac_kernel      four threads (one per wave) per (instance, stage) form the 6 non-trivial Jacobian columns (phi,
//                   vx, vy, omega, d, delta) by central differences and write A_k, B_k, g_k to the
//                   workspace as [B,N,36], [B,N,12], [B,N,6] (read back by the solve kernel).
// Columns X, Y are exactly zero (f does not read X, Y: the reference's f(x+dx) - f(x-dx) is 0.0) and
// are not evaluated.  The difference quotients reuse the parts of f that a perturbation leaves
// unchanged (the tire forces for a phi or d step, the rear force and sin/cos(phi) for a delta step,
// sin/cos(phi) and sin/cos(delta) for vx / vy / omega steps): each reused value is the one f would
// recompute from identical inputs, so the quotients equal the full evaluations.  The shared parts
// are formed from the unperturbed state as the state columns see it (x_i + 0.0, the reference's
// x + dx); the input columns, where the reference passes x itself, see the same values unless a
// component is exactly -0.0 -- then those two columns are evaluated on the exact vectors.
#pragma once
#include "mpc_common.h"

namespace tgmpc {

constexpr double DQ_INV = 1.0 / (2.0 * 1e-5);   // 1 / (2 eps), rounded: the central differences' cdiv

// f of the nominal rollout (mpc_6stati.py:55-71 with the tire model of :25-53); the Pacejka sine is pm_tire_sin,
// as on every path.
__device__ __forceinline__ void rollout_f(const VP& p, const double* x, double d, double delta, double sd, double cd,
                                          double* xd) {
    const double phi = x[2], vx = x[3], vy = x[4], omega = x[5];
    const double avx = fabs(vx);
    const double mx = (p.vx_zero > avx) ? p.vx_zero : avx;
    const double vx_eff = np_sign(vx) * mx;
    const double alpha_f = clampd(-pm_atan2(omega * p.lf + vy, vx_eff) + delta, -p.maxAlpha, p.maxAlpha);
    const double alpha_r = clampd(pm_atan2(omega * p.lr - vy, vx_eff), -p.maxAlpha, p.maxAlpha);
    double sphi, cphi;
    const double sf = pm_tire_sin(p.Cf * pm_atan(p.Bf * alpha_f));
    const double sr = pm_tire_sin(p.Cr * pm_atan(p.Br * alpha_r));
    pm_sincos(phi, &sphi, &cphi);
    const double Fy_f = p.Df * sf, Fy_r = p.Dr * sr;
    const double Frx = (p.Cm1 - p.Cm2 * vx) * d - p.Cr0 - p.Cr2 * (vx * vx);
    xd[0] = vx * cphi - vy * sphi;
    xd[1] = vx * sphi + vy * cphi;
    xd[2] = omega;
    xd[3] = (1.0 / p.m) * (Frx - Fy_f * sd + p.m * vy * omega);
    xd[4] = (1.0 / p.m) * (Fy_r + Fy_f * cd - p.m * vx * omega);
    xd[5] = (1.0 / p.Iz) * (Fy_f * p.lf * cd - Fy_r * p.lr);
}

template <bool CLOSED>
__global__ __launch_bounds__(64) void rollout_kernel(const KArgs a) {
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= a.B) return;
    const traj_vehicle_params& p = a.p;
    const int N = a.c.N;
    const double Ts = a.c.Ts;
    const double* xs = CLOSED ? a.x_state + 6 * (size_t)b : a.x0 + 6 * (size_t)b;
    const double* us = CLOSED ? a.u_state + 2 * (size_t)b : a.u_prev + 2 * (size_t)b;
    double x[6], f[6];
    for (int i = 0; i < 6; ++i) x[i] = xs[i];
    const double u0 = us[0], u1 = us[1];
    double sd, cd;
    pm_sincos(u1, &sd, &cd);
    double* rec = a.wsXF + (size_t)b * N * 12;
    for (int k = 0; k < N; ++k) {
        rollout_f(p, x, u0, u1, sd, cd, f);
        for (int i = 0; i < 6; ++i) {
            rec[12 * k + i] = x[i];
            rec[12 * k + 6 + i] = f[i];
            x[i] = x[i] + Ts * f[i];
        }
    }
}

// parts of the tire model (mpc_6stati.py:25-53), split so perturbations can reuse them
struct Tire {
    double vx_eff, atf, atr;   // vx_eff, atan2(omega lf + vy, vx_eff), atan2(omega lr - vy, vx_eff)
};
__device__ __forceinline__ Tire tire_angles(const VP& p, double vx, double vy, double omega) {
    Tire r;
    const double avx = fabs(vx);
    const double mx = (p.vx_zero > avx) ? p.vx_zero : avx;
    r.vx_eff = np_sign(vx) * mx;
    r.atf = pm_atan2(omega * p.lf + vy, r.vx_eff);
    r.atr = pm_atan2(omega * p.lr - vy, r.vx_eff);
    return r;
}
// The Pacejka sine (physics.h: pm_tire_sin, the same value on every path).
__device__ __forceinline__ double tire_sin(double z) { return pm_tire_sin(z); }
__device__ __forceinline__ double front_force(const VP& p, double atf, double delta) {
    const double alpha_f = clampd(-atf + delta, -p.maxAlpha, p.maxAlpha);
    return p.Df * tire_sin(p.Cf * pm_atan(p.Bf * alpha_f));
}
__device__ __forceinline__ double rear_force(const VP& p, double atr) {
    const double alpha_r = clampd(atr, -p.maxAlpha, p.maxAlpha);
    return p.Dr * tire_sin(p.Cr * pm_atan(p.Br * alpha_r));
}
__device__ __forceinline__ double long_force(const VP& p, double vx, double d) {
    return (p.Cm1 - p.Cm2 * vx) * d - p.Cr0 - p.Cr2 * (vx * vx);
}
// mpc_6stati.py:55-71 from its parts
__device__ __forceinline__ void f_parts(const VP& p, double vx, double vy, double omega, double sphi, double cphi,
                                        double sd, double cd, double Fy_f, double Fy_r, double Frx, double* xd) {
    xd[0] = vx * cphi - vy * sphi;
    xd[1] = vx * sphi + vy * cphi;
    xd[2] = omega;
    xd[3] = (1.0 / p.m) * (Frx - Fy_f * sd + p.m * vy * omega);
    xd[4] = (1.0 / p.m) * (Fy_r + Fy_f * cd - p.m * vx * omega);
    xd[5] = (1.0 / p.Iz) * (Fy_f * p.lf * cd - Fy_r * p.lr);
}
// full f at a state/input point with shared sin/cos
__device__ __forceinline__ void f_full(const VP& p, double vx, double vy, double omega, double sphi, double cphi,
                                       double d, double delta, double sd, double cd, double* xd) {
    const Tire tr = tire_angles(p, vx, vy, omega);
    f_parts(p, vx, vy, omega, sphi, cphi, sd, cd, front_force(p, tr.atf, delta), rear_force(p, tr.atr),
            long_force(p, vx, d), xd);
}

// Jacobian column of state `grp` (0 vx, 1 vy, 2 omega) at rollout point xb with input (d, de), by
// central differences on full f evaluations (one code path for the three columns: the perturbed
// component is selected, the others are the reference's x_i + 0.0).
__device__ __forceinline__ void state_column(const VP& p, const double* xb, double d, double de, int grp, double* J) {
    const double eps = 1e-5;
    const double phi = xb[2] + 0.0, vx = xb[3] + 0.0, vy = xb[4] + 0.0, om = xb[5] + 0.0;
    double sphi, cphi, sd, cd;
    pm_sincos(phi, &sphi, &cphi);
    pm_sincos(de, &sd, &cd);
    double fp[6], fm[6];
    f_full(p, grp == 0 ? xb[3] + eps : vx, grp == 1 ? xb[4] + eps : vy, grp == 2 ? xb[5] + eps : om, sphi, cphi, d,
           de, sd, cd, fp);
    f_full(p, grp == 0 ? xb[3] - eps : vx, grp == 1 ? xb[4] - eps : vy, grp == 2 ? xb[5] - eps : om, sphi, cphi, d,
           de, sd, cd, fm);
    for (int r = 0; r < 6; ++r) J[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
}

// The phi, d and delta columns (Jphi, Jd, Jde), which reuse the base tire evaluation.
__device__ __forceinline__ void cheap_columns(const VP& p, const double* xb, double d, double de, double* Jphi,
                                              double* Jd, double* Jde) {
    const double eps = 1e-5;
    const double phi = xb[2] + 0.0, vx = xb[3] + 0.0, vy = xb[4] + 0.0, om = xb[5] + 0.0;
    double sphi, cphi, sd, cd;
    pm_sincos(phi, &sphi, &cphi);
    pm_sincos(de, &sd, &cd);
    double fp[6], fm[6];
    const Tire t0 = tire_angles(p, vx, vy, om);
    const double Ff0 = front_force(p, t0.atf, de), Fr0 = rear_force(p, t0.atr), Fx0 = long_force(p, vx, d);
    {   // phi: only sin/cos(phi) change
        double sp, cp, sm, cm;
        pm_sincos(xb[2] + eps, &sp, &cp);
        pm_sincos(xb[2] - eps, &sm, &cm);
        f_parts(p, vx, vy, om, sp, cp, sd, cd, Ff0, Fr0, Fx0, fp);
        f_parts(p, vx, vy, om, sm, cm, sd, cd, Ff0, Fr0, Fx0, fm);
        for (int r = 0; r < 6; ++r) Jphi[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
    }
    {   // d: only the longitudinal force changes
        f_parts(p, vx, vy, om, sphi, cphi, sd, cd, Ff0, Fr0, long_force(p, vx, d + eps), fp);
        f_parts(p, vx, vy, om, sphi, cphi, sd, cd, Ff0, Fr0, long_force(p, vx, d - eps), fm);
        for (int r = 0; r < 6; ++r) Jd[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
    }
    {   // delta: front force and sin/cos(delta) change
        double sp, cp, sm, cm;
        pm_sincos(de + eps, &sp, &cp);
        pm_sincos(de - eps, &sm, &cm);
        f_parts(p, vx, vy, om, sphi, cphi, sp, cp, front_force(p, t0.atf, de + eps), Fr0, Fx0, fp);
        f_parts(p, vx, vy, om, sphi, cphi, sm, cm, front_force(p, t0.atf, de - eps), Fr0, Fx0, fm);
        for (int r = 0; r < 6; ++r) Jde[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
    }
    // a -0.0 among the components the input columns pass through: evaluate those two columns on
    // the reference's exact vectors, f(x, u +- du) with u_other + 0.0 (signed zeros match too)
    if ((__builtin_signbit(xb[2]) && xb[2] == 0.0) || (__builtin_signbit(xb[3]) && xb[3] == 0.0) ||
        (__builtin_signbit(xb[4]) && xb[4] == 0.0) || (__builtin_signbit(xb[5]) && xb[5] == 0.0) ||
        (__builtin_signbit(d) && d == 0.0) || (__builtin_signbit(de) && de == 0.0)) {
        for (int cu = 0; cu < 2; ++cu) {
            const double up[2] = {cu == 0 ? d + eps : d + 0.0, cu == 1 ? de + eps : de + 0.0};
            const double um[2] = {cu == 0 ? d - eps : d + 0.0, cu == 1 ? de - eps : de + 0.0};
            double xc[6];
            for (int i = 0; i < 6; ++i) xc[i] = xb[i];
            f_cont(p, xc, up, fp);
            f_cont(p, xc, um, fm);
            for (int r = 0; r < 6; ++r) (cu == 0 ? Jd : Jde)[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
        }
    }
}

// :106-108 for one stage: A = I + Ts Jx, B = Ts Ju (columns X, Y of Jx exactly zero)
__device__ __forceinline__ double a_entry(int r, int cc, double Ts, double Jrc) {
    return ((r == cc) ? 1.0 : 0.0) + Ts * Jrc;
}
// g = x + Ts f - A x - B u  (f = the rollout's f(x_k, u))
__device__ __forceinline__ void g_stage(const double* A, const double* Bm, const double* xb, const double* fk, double d,
                                       double de, double Ts, double* g) {
    for (int r = 0; r < 6; ++r) {
        double ax = 0.0, bu = 0.0;
        for (int cc = 0; cc < 6; ++cc) ax += A[6 * r + cc] * xb[cc];
        bu += Bm[2 * r] * d;
        bu += Bm[2 * r + 1] * de;
        g[r] = xb[r] + Ts * fk[r] - ax - bu;
    }
}

// One workgroup = 4 waves x 64 stages: waves 0-2 form the vx / vy / omega columns of their 64
// stages (a full tire evaluation per side), wave 3 the base tire and the cheap phi / d / delta
// columns, then assembles A_k, B_k, g_k from the columns staged in LDS (wave-uniform branches).
template <bool CLOSED>
__global__ __launch_bounds__(256) void jac_kernel(const KArgs a) {
    __shared__ double sJ[64][6][6];   // [stage in block][column - 2][row]
    const int N = a.c.N;
    const int s = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int gs = blockIdx.x * 64 + s;
    const bool valid = gs < a.B * N;
    const int b = valid ? gs / N : 0, k = valid ? gs - b * N : 0;
    const traj_vehicle_params& p = a.p;
    const double Ts = a.c.Ts;
    const double* rec = a.wsXF + ((size_t)b * N + k) * 12;
    const double* us = CLOSED ? a.u_state + 2 * (size_t)b : a.u_prev + 2 * (size_t)b;
    double xb[6];
    for (int i = 0; i < 6; ++i) xb[i] = valid ? rec[i] : 0.0;
    const double d = valid ? us[0] : 0.0, de = valid ? us[1] : 0.0;
    double (*J)[6] = sJ[s];
    if (grp < 3) state_column(p, xb, d, de, grp, J[1 + grp]);   // vx, vy, omega
    else cheap_columns(p, xb, d, de, J[0], J[4], J[5]);        // phi, d, delta
    __syncthreads();
    if (grp != 3 || !valid) return;
    // :106-108  A = I + Ts Jx ; B = Ts Ju ; g = x + Ts f - A x - B u   (f = the rollout's f(x_k, u))
    double A[36], Bm[12], g[6];
    for (int r = 0; r < 6; ++r) {
        A[6 * r + 0] = a_entry(r, 0, Ts, 0.0);
        A[6 * r + 1] = a_entry(r, 1, Ts, 0.0);
        for (int cc = 2; cc < 6; ++cc) A[6 * r + cc] = a_entry(r, cc, Ts, J[cc - 2][r]);
        Bm[2 * r + 0] = Ts * J[4][r];
        Bm[2 * r + 1] = Ts * J[5][r];
    }
    g_stage(A, Bm, xb, rec + 6, d, de, Ts, g);
    const size_t o = (size_t)b * N + k;
    double* wA = a.wsA + o * 36;
    double* wB = a.wsB + o * 12;
    double* wg = a.wsg + o * 6;
    for (int i = 0; i < 36; ++i) wA[i] = A[i];
    for (int i = 0; i < 12; ++i) wB[i] = Bm[i];
    for (int r = 0; r < 6; ++r) wg[r] = g[r];
}

// In-workgroup linearization for the fused closed loop (traj_closed_loop_run): rollout_kernel's
// and jac_kernel's arithmetic for ONE instance and NT threads, with A_k, B_k, g_k written to LDS in the
// stage records the solve kernel's condensing reads.  xs / us: the state and input (LDS).  Ends with a barrier.
//
// The rollout is a serial chain through the tire forces: per stage, atan2 -> atan -> the Pacejka sine on two lanes.
// Only vx, vy and omega feed back (f_3..5 do not read X, Y or phi; phi_{k+1} = phi_k + Ts omega_k), so the chain
// carries those and phi; sin / cos(phi_k) -- needed only for X, Y and the phi column -- are evaluated after it, for
// all stages at once, and X_k, Y_k are then summed in the rollout's order.  The Jacobian columns of stage k need
// the tire chain at perturbed copies of x_k, known as soon as x_k is: lanes 3 .. 18 run those evaluations IN THE
// SAME instruction stream as the rollout lanes (the stage's latency does not change).  Lane roles, stage k:
//   0 / 1       rollout: front tire, rear tire at x_k (raw, rollout_kernel's form)
//   3 / 4       base front / rear tire at x_k + 0.0 (cheap_columns' t0)
//   5 .. 16     4 lanes per state column (vx, vy, omega): (+eps front, +eps rear, -eps front, -eps rear)
//   17 / 18     front tire at delta +- eps (the delta column)
// Their sines go to tj[k][lane].  The phi pass (after the chain), lane v N + k: sincos(phi_k + {-0.0, +eps, -eps}),
// v = 0 / 1 / 2: sin / cos(phi_k + 0.0) -> tj[k][21] / tj[k][2] (sin(phi + 0.0) = sin(phi) + 0.0 exactly, cos is
// even), sin / cos(phi_k +- eps) -> tj[k][19 / 20] / tj[k][0 / 1], and lane k forms the rollout's f_0, f_1 of stage
// k from the raw sin / cos.  An assembly pass (one stage per lane) then forms f at each perturbed point with f_parts
// and the difference quotients: the values state_column / cheap_columns compute (jac_kernel), bit for bit.
constexpr int TJ = 24;
// Layout: one record of LREC doubles per stage, rec + LREC k = [A_k 36 | B_k 12 | g_k 6] on exit.  While
// the stage is being formed the same record holds its scratch: the tire / sincos evaluations at [0, TJ) and
// the rollout's (x_k, f_k) at [TJ, TJ + 12).  Only the lane that assembles stage k reads them, and it writes
// the outputs after its reads, so no stage's scratch is overwritten before it is consumed.
constexpr int LREC = 54;
static_assert(TJ + 12 <= 36, "a stage's scratch must lie inside its record's A_k part");
template <int NT>
__device__ __forceinline__ void block_linearize(const int t, const VP& p, int N, double Ts, const double* xs,
                                                const double* us, double* rec, long long* dbg = nullptr) {
    double* const tj = rec;                // [k]: rec + LREC k + [0, TJ)
    double* const xf = rec + TJ;           // [k]: rec + LREC k + TJ + [0, 12)
    auto mark = [&](int i) { if (dbg && t == 0) dbg[i] = __builtin_amdgcn_s_memtime(); };
    const double eps = 1e-5;
    if (t < 64) {
        double x[6];
        for (int i = 2; i < 6; ++i) x[i] = xs[i];
        const double u0 = us[0], u1 = us[1];
        double sd, cd;
        pm_sincos(u1, &sd, &cd);
        // this lane's role (see above): which tire, which input it perturbs
        const bool roll = t < 2;
        const bool fr = (t == 0) || (t == 3) || (t >= 5 && t <= 16 && ((t - 5) & 1) == 0) || t == 17 || t == 18;
        const int col = (t >= 5 && t <= 16) ? (t - 5) >> 2 : -1;             // 0 vx, 1 vy, 2 omega
        const double sgn = (t >= 5 && t <= 16 && ((t - 5) & 2)) ? -eps : eps;
        const double dlt = (t == 17) ? u1 + eps : ((t == 18) ? u1 - eps : u1);
        const double Bt = fr ? p.Bf : p.Br, Ct = fr ? p.Cf : p.Cr;
        // The roles as per-lane constants, so the stage body is one branch-free instruction stream: the
        // evaluation point is x_i + d_i with d_i = -0.0 on the rollout lanes (x + -0.0 = x for every x, -0.0
        // included), 0.0 for the base evaluations (x_i + 0.0) and +-eps for a column's perturbed component; the
        // rear tire's "oml lr - vyl" as oml lr + (-1 vyl) and its alpha "at" as 1 at + -0.0 (exact identities)
        const double dvx = roll ? -0.0 : (col == 0 ? sgn : 0.0);
        const double dvy = roll ? -0.0 : (col == 1 ? sgn : 0.0);
        const double dom = roll ? -0.0 : (col == 2 ? sgn : 0.0);
        const double Lt = fr ? p.lf : p.lr, sy = fr ? 1.0 : -1.0, sa = fr ? -1.0 : 1.0, dl = fr ? dlt : -0.0;
        // lanes whose sine is used (the range check of the Pacejka sine's fast form looks at these only)
        const unsigned long long used = 0x7fffbull;   // lanes 0, 1, 3 .. 18
        for (int k = 0; k < N; ++k) {
            const double phi = x[2], vx = x[3], vy = x[4], omega = x[5];
            // this lane's evaluation point (state_column / cheap_columns: x_i + 0.0, the column x_i +- eps)
            const double vxl = vx + dvx, vyl = vy + dvy, oml = omega + dom;
            const double avx = fabs(vxl);
            const double mx = (p.vx_zero > avx) ? p.vx_zero : avx;
            const double vx_eff = np_sign(vxl) * mx;
            const double at = pm_atan2(oml * Lt + sy * vyl, vx_eff);
            const double alpha = clampd(sa * at + dl, -p.maxAlpha, p.maxAlpha);
            const double z = Ct * pm_atan(Bt * alpha);
            // pm_tire_sin per lane: the polynomial, or -- where a used lane's argument leaves its interval (other
            // Params, NaN) -- the library sine on those lanes (a wave-uniform branch around it)
            double sz = tire_sin_poly(z);
            if (__ballot(!tire_sin_in_range(z)) & used) {
                if (!tire_sin_in_range(z)) sz = pm_sin(z);
            }
            if (t >= 3 && t <= 18) tj[LREC * k + t] = sz;
            const double Fy_f = p.Df * readlane_d(sz, 0), Fy_r = p.Dr * readlane_d(sz, 1);
            const double Frx = (p.Cm1 - p.Cm2 * vx) * u0 - p.Cr0 - p.Cr2 * (vx * vx);
            double f[6];
            f[2] = omega;
            f[3] = (1.0 / p.m) * (Frx - Fy_f * sd + p.m * vy * omega);
            f[4] = (1.0 / p.m) * (Fy_r + Fy_f * cd - p.m * vx * omega);
            f[5] = (1.0 / p.Iz) * (Fy_f * p.lf * cd - Fy_r * p.lr);
            if (t == 0)
                for (int i = 2; i < 6; ++i) {
                    xf[LREC * k + i] = x[i];
                    xf[LREC * k + 6 + i] = f[i];
                }
            for (int i = 2; i < 6; ++i) x[i] = x[i] + Ts * f[i];
            (void)phi;
        }
    }
    __syncthreads();
    // the phi pass: lane v N + k, stage k, offset {-0.0, +eps, -eps}[v] (3 N <= 64 lanes per round)
    for (int l = t; l < 3 * N; l += NT) {
        const int v = l / N, k = l - v * N;
        const double phik = xf[LREC * k + 2];
        double sp, cp;
        pm_sincos(phik + (v == 0 ? -0.0 : (v == 1 ? eps : -eps)), &sp, &cp);
        double* const T = tj + LREC * k;
        if (v == 0) {
            T[21] = sp + 0.0;   // sin(phi + 0.0)
            T[2] = cp;          // cos(phi + 0.0)
            const double vx = xf[LREC * k + 3], vy = xf[LREC * k + 4];
            xf[LREC * k + 6] = vx * cp - vy * sp;   // the rollout's f_0, f_1 at the raw phi_k
            xf[LREC * k + 7] = vx * sp + vy * cp;
        } else {
            T[18 + v] = sp;     // 19: phi + eps, 20: phi - eps
            T[v - 1] = cp;      // 0 / 1
        }
    }
    __syncthreads();
    // X_k, Y_k in the rollout's order: X_{k+1} = X_k + Ts f_0(x_k)
    if (t == 0) {
        double X = xs[0], Y = xs[1];
        for (int k = 0; k < N; ++k) {
            xf[LREC * k + 0] = X;
            xf[LREC * k + 1] = Y;
            X = X + Ts * xf[LREC * k + 6];
            Y = Y + Ts * xf[LREC * k + 7];
        }
    }
    __syncthreads();
    mark(20);
    mark(21);
    const double d = us[0], de = us[1];
    // assembly: one stage per lane -- f at every perturbed point from the stored sines (f_parts, the
    // reference's difference quotients), A = I + Ts Jx, B = Ts Ju, g = x + Ts f - A x - B u
    double sd, cd, sdp, cdp, sdm, cdm;
    pm_sincos(de, &sd, &cd);
    pm_sincos(de + eps, &sdp, &cdp);
    pm_sincos(de - eps, &sdm, &cdm);
    for (int k = t; k < N; k += NT) {
        const double* T = tj + LREC * k;
        double xb[6], fk[6];
        for (int i = 0; i < 6; ++i) { xb[i] = xf[LREC * k + i]; fk[i] = xf[LREC * k + 6 + i]; }
        const double vx0 = xb[3] + 0.0, vy0 = xb[4] + 0.0, om0 = xb[5] + 0.0;
        const double sphi = T[21], cphi = T[2];
        const double Ff0 = p.Df * T[3], Fr0 = p.Dr * T[4], Fx0 = long_force(p, vx0, d);
        double Ak[36], Bk[12], fp[6], fm[6];
        for (int grp = 0; grp < 3; ++grp) {   // state columns (state_column)
            const double vxp = grp == 0 ? xb[3] + eps : vx0, vxm = grp == 0 ? xb[3] - eps : vx0;
            const double vyp = grp == 1 ? xb[4] + eps : vy0, vym = grp == 1 ? xb[4] - eps : vy0;
            const double omp = grp == 2 ? xb[5] + eps : om0, omm = grp == 2 ? xb[5] - eps : om0;
            const int l = 5 + 4 * grp;
            f_parts(p, vxp, vyp, omp, sphi, cphi, sd, cd, p.Df * T[l], p.Dr * T[l + 1], long_force(p, vxp, d), fp);
            f_parts(p, vxm, vym, omm, sphi, cphi, sd, cd, p.Df * T[l + 2], p.Dr * T[l + 3], long_force(p, vxm, d), fm);
            for (int r = 0; r < 6; ++r) Ak[6 * r + 3 + grp] = a_entry(r, 3 + grp, Ts, cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV));
        }
        double Jphi[6], Jd[6], Jde[6];
        // phi: only sin / cos(phi) change
        f_parts(p, vx0, vy0, om0, T[19], T[0], sd, cd, Ff0, Fr0, Fx0, fp);
        f_parts(p, vx0, vy0, om0, T[20], T[1], sd, cd, Ff0, Fr0, Fx0, fm);
        for (int r = 0; r < 6; ++r) Jphi[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
        // d: only the longitudinal force changes
        f_parts(p, vx0, vy0, om0, sphi, cphi, sd, cd, Ff0, Fr0, long_force(p, vx0, d + eps), fp);
        f_parts(p, vx0, vy0, om0, sphi, cphi, sd, cd, Ff0, Fr0, long_force(p, vx0, d - eps), fm);
        for (int r = 0; r < 6; ++r) Jd[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
        // delta: front force and sin / cos(delta) change
        f_parts(p, vx0, vy0, om0, sphi, cphi, sdp, cdp, p.Df * T[17], Fr0, Fx0, fp);
        f_parts(p, vx0, vy0, om0, sphi, cphi, sdm, cdm, p.Df * T[18], Fr0, Fx0, fm);
        for (int r = 0; r < 6; ++r) Jde[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
        // a -0.0 among the components the input columns pass through: those two columns on the
        // reference's exact vectors, as cheap_columns does
        if ((__builtin_signbit(xb[2]) && xb[2] == 0.0) || (__builtin_signbit(xb[3]) && xb[3] == 0.0) ||
            (__builtin_signbit(xb[4]) && xb[4] == 0.0) || (__builtin_signbit(xb[5]) && xb[5] == 0.0) ||
            (__builtin_signbit(d) && d == 0.0) || (__builtin_signbit(de) && de == 0.0)) {
            for (int cu = 0; cu < 2; ++cu) {
                const double up[2] = {cu == 0 ? d + eps : d + 0.0, cu == 1 ? de + eps : de + 0.0};
                const double um[2] = {cu == 0 ? d - eps : d + 0.0, cu == 1 ? de - eps : de + 0.0};
                double xc[6];
                for (int i = 0; i < 6; ++i) xc[i] = xb[i];
                f_cont(p, xc, up, fp);
                f_cont(p, xc, um, fm);
                for (int r = 0; r < 6; ++r) (cu == 0 ? Jd : Jde)[r] = cdiv(fp[r] - fm[r], 2.0 * eps, DQ_INV);
            }
        }
        for (int r = 0; r < 6; ++r) {
            Ak[6 * r + 0] = a_entry(r, 0, Ts, 0.0);
            Ak[6 * r + 1] = a_entry(r, 1, Ts, 0.0);
            Ak[6 * r + 2] = a_entry(r, 2, Ts, Jphi[r]);
            Bk[2 * r + 0] = Ts * Jd[r];
            Bk[2 * r + 1] = Ts * Jde[r];
        }
        double gk[6];
        g_stage(Ak, Bk, xb, fk, d, de, Ts, gk);
        double* const o = rec + LREC * k;   // (after every read of this stage's scratch)
        for (int i = 0; i < 36; ++i) o[i] = Ak[i];
        for (int i = 0; i < 12; ++i) o[36 + i] = Bk[i];
        for (int r = 0; r < 6; ++r) o[48 + r] = gk[r];
    }
    __syncthreads();
}

}  // namespace tgmpc
