// physics.h -- device restatement of the 6-state dynamic bicycle model of the reference
// (MPC/mpc_6stati.py:21-117).  Compiled with -ffp-contract=off so every expression keeps the
// reference's numpy evaluation order term by term (no FMA contraction); transcendentals come from
// the ROCm device libm (ocml), which can differ from numpy's SIMD libm in the last ulp.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/trajmpc.h"
#include "fastmath.h"

#ifndef TGMPC_FASTMATH
// 1: the MPC path's sincos / atan / atan2 from fastmath.h.  Measured slower (rollout 50.6 k -> 55.4 k cycles per
// item, 12.36 -> 11.99 M steps/s at the driver's command; the per-lane fallback branches and region selects cost
// more than the shorter polynomials save), so the device library's routines stay the default.
#define TGMPC_FASTMATH 0
#endif

namespace tgmpc {

// The transcendentals of the MPC path: every kernel (fused closed loop, per-step launches, physics and window
// entry points) calls these, so all of them evaluate f, the slip angles and the window identically.
__device__ __forceinline__ void pm_sincos(double x, double* s, double* c) {
#if TGMPC_FASTMATH
    fm_sincos(x, s, c);
#else
    sincos(x, s, c);
#endif
}
__device__ __forceinline__ double pm_sin(double x) {
    double s, c;
    pm_sincos(x, &s, &c);
    return s;
}
__device__ __forceinline__ double pm_atan(double x) {
#if TGMPC_FASTMATH
    return fm_atan(x);
#else
    return atan(x);
#endif
}
__device__ __forceinline__ double pm_atan2(double y, double x) {
#if TGMPC_FASTMATH
    return fm_atan2(y, x);
#else
    return atan2(y, x);
#endif
}

typedef traj_vehicle_params VP;

// The Pacejka sine, sin(C atan(B alpha)).  Its argument is bounded: |alpha| <= maxAlpha after the clamp, so
// |z| <= C atan(B maxAlpha) (1.414 with the reference's Params) -- inside [-pi/2, pi/2], where no argument reduction
// is needed.  There sin is the odd Taylor polynomial through x^21 (the next term is below 2e-18 at pi/2): x + x^3 q(x^2),
// q by Horner with fma, 12 VALU against the ~80 of the library's sincos, within 2 ulp of the correctly rounded sine
// (checked against a 120-bit reference over 4e5 points).  Outside the interval (other Params) and for NaN: the
// library's sine.  Every path of the MPC (fused and per-step linearization, the physics entry points, the plant
// update) evaluates the tire force through this function, so they agree bit for bit.
constexpr double TIRE_SIN_ZMAX = 1.5707963267948966;
__device__ __forceinline__ double tire_sin_poly(double x) {
    const double x2 = x * x;
    double q = 1.9572941063391263e-20;
    q = fma(q, x2, -8.22063524662433e-18);
    q = fma(q, x2, 2.8114572543455206e-15);
    q = fma(q, x2, -7.647163731819816e-13);
    q = fma(q, x2, 1.6059043836821613e-10);
    q = fma(q, x2, -2.505210838544172e-08);
    q = fma(q, x2, 2.7557319223985893e-06);
    q = fma(q, x2, -0.0001984126984126984);
    q = fma(q, x2, 0.008333333333333333);
    q = fma(q, x2, -0.16666666666666666);
    return fma(x2 * x, q, x);
}
__device__ __forceinline__ bool tire_sin_in_range(double z) { return fabs(z) <= TIRE_SIN_ZMAX; }
__device__ __forceinline__ double pm_tire_sin(double z) {
    return tire_sin_in_range(z) ? tire_sin_poly(z) : pm_sin(z);
}

// np.sign: +1 / -1 / +0.0 for both zeros / NaN passes through
__device__ __forceinline__ double np_sign(double x) {
    return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}

// mpc_6stati.py:21-23  np.minimum(np.maximum(x, lo), hi)  (NaN propagates)
__device__ __forceinline__ double clampd(double x, double lo, double hi) {
    double t = (x < lo) ? lo : x;
    return (t > hi) ? hi : t;
}

// mpc_6stati.py:25-53
__device__ __forceinline__ void tire_forces(const VP& p, double vx, double vy, double omega, double d, double delta,
                                            double& Fy_f, double& Fy_r, double& Frx) {
    double avx = fabs(vx);
    double mx = (p.vx_zero > avx) ? p.vx_zero : avx;  // python max(abs(vx), vx_zero)
    double vx_eff = np_sign(vx) * mx;
    double alpha_f = -pm_atan2(omega * p.lf + vy, vx_eff) + delta;
    double alpha_r = pm_atan2(omega * p.lr - vy, vx_eff);
    alpha_f = clampd(alpha_f, -p.maxAlpha, p.maxAlpha);
    alpha_r = clampd(alpha_r, -p.maxAlpha, p.maxAlpha);
    Fy_f = p.Df * pm_tire_sin(p.Cf * pm_atan(p.Bf * alpha_f));
    Fy_r = p.Dr * pm_tire_sin(p.Cr * pm_atan(p.Br * alpha_r));
    Frx = (p.Cm1 - p.Cm2 * vx) * d - p.Cr0 - p.Cr2 * (vx * vx);
}

// mpc_6stati.py:55-71.  sd/cd = sin/cos(delta) may be supplied (they only depend on u).
__device__ __forceinline__ void f_cont_sc(const VP& p, const double* x, double d, double delta, double sd, double cd,
                                          double* xd) {
    double phi = x[2], vx = x[3], vy = x[4], omega = x[5];
    double Fy_f, Fy_r, Frx;
    tire_forces(p, vx, vy, omega, d, delta, Fy_f, Fy_r, Frx);
    double sphi, cphi;
    pm_sincos(phi, &sphi, &cphi);
    xd[0] = vx * cphi - vy * sphi;
    xd[1] = vx * sphi + vy * cphi;
    xd[2] = omega;
    xd[3] = (1.0 / p.m) * (Frx - Fy_f * sd + p.m * vy * omega);
    xd[4] = (1.0 / p.m) * (Fy_r + Fy_f * cd - p.m * vx * omega);
    xd[5] = (1.0 / p.Iz) * (Fy_f * p.lf * cd - Fy_r * p.lr);
}

__device__ __forceinline__ void f_cont(const VP& p, const double* x, const double* u, double* xd) {
    double sd, cd;
    pm_sincos(u[1], &sd, &cd);
    f_cont_sc(p, x, u[0], u[1], sd, cd, xd);
}

// mpc_6stati.py:111-117
__device__ __forceinline__ double lateral_error(double X, double Y, double Xr, double Yr, double phir) {
    double s, c;
    pm_sincos(phir, &s, &c);
    return s * (X - Xr) - c * (Y - Yr);
}

}  // namespace tgmpc
