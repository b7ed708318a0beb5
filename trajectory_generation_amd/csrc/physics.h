// physics.h -- device restatement of the 6-state dynamic bicycle model of the reference
// (MPC/mpc_6stati.py:21-117).  Compiled with -ffp-contract=off so every expression keeps the
// reference's numpy evaluation order term by term (no FMA contraction); transcendentals come from
// the ROCm device libm (ocml), which can differ from numpy's SIMD libm in the last ulp.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/trajmpc.h"

namespace tgmpc {

typedef traj_vehicle_params VP;

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
    double alpha_f = -atan2(omega * p.lf + vy, vx_eff) + delta;
    double alpha_r = atan2(omega * p.lr - vy, vx_eff);
    alpha_f = clampd(alpha_f, -p.maxAlpha, p.maxAlpha);
    alpha_r = clampd(alpha_r, -p.maxAlpha, p.maxAlpha);
    Fy_f = p.Df * sin(p.Cf * atan(p.Bf * alpha_f));
    Fy_r = p.Dr * sin(p.Cr * atan(p.Br * alpha_r));
    Frx = (p.Cm1 - p.Cm2 * vx) * d - p.Cr0 - p.Cr2 * (vx * vx);
}

// mpc_6stati.py:55-71.  sd/cd = sin/cos(delta) may be supplied (they only depend on u).
__device__ __forceinline__ void f_cont_sc(const VP& p, const double* x, double d, double delta, double sd, double cd,
                                          double* xd) {
    double phi = x[2], vx = x[3], vy = x[4], omega = x[5];
    double Fy_f, Fy_r, Frx;
    tire_forces(p, vx, vy, omega, d, delta, Fy_f, Fy_r, Frx);
    double sphi, cphi;
    sincos(phi, &sphi, &cphi);
    xd[0] = vx * cphi - vy * sphi;
    xd[1] = vx * sphi + vy * cphi;
    xd[2] = omega;
    xd[3] = (1.0 / p.m) * (Frx - Fy_f * sd + p.m * vy * omega);
    xd[4] = (1.0 / p.m) * (Fy_r + Fy_f * cd - p.m * vx * omega);
    xd[5] = (1.0 / p.Iz) * (Fy_f * p.lf * cd - Fy_r * p.lr);
}

__device__ __forceinline__ void f_cont(const VP& p, const double* x, const double* u, double* xd) {
    double sd, cd;
    sincos(u[1], &sd, &cd);
    f_cont_sc(p, x, u[0], u[1], sd, cd, xd);
}

// mpc_6stati.py:111-117
__device__ __forceinline__ double lateral_error(double X, double Y, double Xr, double Yr, double phir) {
    double s, c;
    sincos(phir, &s, &c);
    return s * (X - Xr) - c * (Y - Yr);
}

}  // namespace tgmpc
