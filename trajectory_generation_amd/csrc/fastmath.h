// fastmath.h -- float64 sincos / atan / atan2 for the MPC path, with a fraction of the instructions (and of the
// dependent depth) of the general-purpose device library routines.
//
// The rollout of the nominal trajectory (mpc_6stati.py:165-172) and the central-difference linearization
// (:73-109) evaluate atan2 -> atan -> sin per tire and sin / cos(phi) per stage; in the fused closed loop that
// chain is ~20 % of a work item's instructions.  These routines:
//   * fm_sincos: x = n pi/2 + r with n = rint(x 2/pi) and r = fma(-n, PIO2_HI, x) (exact for |n| < 2^20: both
//     terms are multiples of 2^-53 and |r| <= pi/4) minus n PIO2_MID, its rounding kept as a tail; the kernel
//     polynomials of FreeBSD's k_sin.c / k_cos.c with that tail (|r| <= pi/4, < 1 ulp), quadrant by n mod 4.  |x| >= 2^20 pi/2 or non-finite: the device
//     library's sincos for that lane.
//   * fm_atan: |x| reduced to |r| <= 7/16 in three regions -- r = |x| (|x| <= 7/16); r = (|x| - 1) / (|x| + 1),
//     offset pi/4 (<= 39/16); r = -1 / |x|, offset pi/2 -- with ONE division (v_rcp_f64 + 2 Newton steps + one
//     residual correction), then FreeBSD s_atan.c's odd polynomial (11 terms, |r| <= 7/16) and its hi / lo
//     offset sum.
//   * fm_atan2: the same core on the pair (|y|, |x|) (no rounded quotient y / x first), then the quadrant;
//     non-finite or (0, 0) arguments take the device library's atan2 for that lane.
// Accuracy against 80-bit references (tools/microbench/fastmath_check.hip, 4 M points per range on the GPU): see
// DESIGN.md (the device library's own routines: 0.8 ulp sin / cos, 1.5 atan, 1.6 atan2).  The reference path's own functions are numpy's (glibc):
// the physics fixtures are checked at 1e-12 relative and the difference quotients at 1e-8 (tests/).
// Every caller in the MPC path (fused and per-step kernels, the physics entry points, the window kernels) uses
// these, so the fused closed loop and the per-step launches stay bit-identical.
#pragma once
#include <hip/hip_runtime.h>

namespace tgmpc {

namespace fmk {
// FreeBSD msun k_sin.c / k_cos.c / s_atan.c coefficients (public domain, Sun Microsystems 1993)
constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                 C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                 C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
constexpr double AT0 = 3.33333333333329318027e-01, AT1 = -1.99999999998764832476e-01,
                 AT2 = 1.42857142725034663711e-01, AT3 = -1.11111104054623557880e-01,
                 AT4 = 9.09088713343650656196e-02, AT5 = -7.69187620504482999495e-02,
                 AT6 = 6.66107313738753120669e-02, AT7 = -5.83357013379057348645e-02,
                 AT8 = 4.97687799461593236017e-02, AT9 = -3.65315727442169155270e-02,
                 AT10 = 1.62858201153657823623e-02;
constexpr double PIO4_HI = 7.85398163397448278999e-01, PIO4_LO = 3.06161699786838301793e-17;
constexpr double PIO2_HI = 1.57079632679489655800e+00, PIO2_LO = 6.12323399573676603587e-17;
constexpr double PI_HI = 3.1415926535897931160e+00, PI_LO = 1.2246467991473531772e-16;
constexpr double TWO_OVER_PI = 6.36619772367581382433e-01;
constexpr double PIO2_MID = 6.123233995736766035868820147291818e-17;   // pi/2 - PIO2_HI
constexpr double SC_LIMIT = 1647099.3291652855;   // 2^20 pi / 2

__device__ __forceinline__ double flip(double v, bool neg) {   // v or -v (sign bit)
    return neg ? -v : v;
}
// sin(r + y), cos(r + y) for |r| <= pi/4, y the reduction's tail (k_sin.c / k_cos.c)
__device__ __forceinline__ void kernel_sincos(double r, double y, double& s, double& c) {
    const double z = r * r, w = z * z;
    const double rs = fma(z, fma(z, S4, S3), S2) + z * w * fma(z, S6, S5);
    const double v = z * r;
    s = r - ((z * (0.5 * y - v * rs) - y) - v * S1);
    const double rc = z * fma(z, fma(z, C3, C2), C1) + w * w * fma(z, fma(z, C6, C5), C4);
    const double hz = 0.5 * z, wc = 1.0 - hz;
    c = wc + (((1.0 - wc) - hz) + (z * rc - r * y));
}
// atan(num / den) for a reduced pair with |num / den| <= 7/16 (den >= 1), plus offset (hi, lo):
// off_hi - ((r s - off_lo) - r) as s_atan.c
__device__ __forceinline__ double atan_core(double num, double den, double off_hi, double off_lo) {
    double rc = __builtin_amdgcn_rcp(den);
    rc = fma(fma(-den, rc, 1.0), rc, rc);
    rc = fma(fma(-den, rc, 1.0), rc, rc);
    const double q = num * rc;
    const double r = fma(fma(-den, q, num), rc, q);
    const double z = r * r, w = z * z;
    const double s1 = z * fma(w, fma(w, fma(w, fma(w, fma(w, AT10, AT8), AT6), AT4), AT2), AT0);
    const double s2 = w * fma(w, fma(w, fma(w, fma(w, AT9, AT7), AT5), AT3), AT1);
    return off_hi - ((r * (s1 + s2) - off_lo) - r);
}
// atan(a / b) for a, b >= 0 (b > 0 or a > 0, both finite): region by the ratio, one division
__device__ __forceinline__ double atan_pos(double a, double b) {
    const bool big = a > 2.4375 * b;                 // ratio > 39/16: r = -b / a, offset pi/2
    const bool mid = !big && a > 0.4375 * b;         // 7/16 < ratio <= 39/16: r = (a - b) / (a + b), offset pi/4
    const double num = big ? -b : (mid ? a - b : a);
    double den = big ? a : (mid ? a + b : b);
    den = fmin(den, 0x1p+1000);                      // (a huge a: the quotient is 0 to the result's precision)
    const double oh = big ? PIO2_HI : (mid ? PIO4_HI : 0.0);
    const double ol = big ? PIO2_LO : (mid ? PIO4_LO : 0.0);
    return atan_core(num, den, oh, ol);
}
}  // namespace fmk

// sin and cos of x
__device__ __forceinline__ void fm_sincos(double x, double* sp, double* cp) {
    const double ax = fabs(x);
    if (!(ax < fmk::SC_LIMIT)) {   // huge or non-finite: the library routine (rare, per lane)
        sincos(x, sp, cp);
        return;
    }
    const double n = rint(x * fmk::TWO_OVER_PI);
    const double r1 = fma(-n, fmk::PIO2_HI, x);                 // exact (see above)
    const double r = fma(-n, fmk::PIO2_MID, r1);
    const double y = fma(-n, fmk::PIO2_MID, r1 - r);            // the rounding of r (the pi/2 tail past MID is < 1e-32 n)
    double s, c;
    fmk::kernel_sincos(r, y, s, c);
    const int q = (int)n & 3;
    const bool swap = q & 1;
    *sp = fmk::flip(swap ? c : s, q & 2);
    *cp = fmk::flip(swap ? s : c, q == 1 || q == 2);
}

__device__ __forceinline__ double fm_sin(double x) {
    double s, c;
    fm_sincos(x, &s, &c);
    return s;
}

// atan(x)
__device__ __forceinline__ double fm_atan(double x) {
    const double r = fmk::atan_pos(fabs(x), 1.0);
    return copysign(r, x);   // (NaN in, NaN out)
}

// atan2(y, x)
__device__ __forceinline__ double fm_atan2(double y, double x) {
    const double ay = fabs(y), ax = fabs(x);
    if (!(ax < INFINITY && ay < INFINITY) || (ax == 0.0 && ay == 0.0)) return atan2(y, x);   // per lane, rare
    double r = fmk::atan_pos(ay, ax);                 // in [0, pi/2]
    if (__builtin_signbit(x)) r = fmk::PI_HI - (r - fmk::PI_LO);
    return copysign(r, y);
}

}  // namespace tgmpc
