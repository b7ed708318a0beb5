// Accuracy of fastmath.h (fm_sincos / fm_atan / fm_atan2) and of the device library's routines against x87
// 80-bit references (sinl, cosl, atanl, atan2l) on the host: max and mean error in ulps of the double result,
// per argument range (the MPC path's ranges and wider ones).  Also checks the special cases.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "../../trajectory_generation_amd/csrc/fastmath.h"

using namespace tgmpc;

__global__ void eval(const double* x, const double* y, double* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double s, c, s2, c2;
    fm_sincos(x[i], &s, &c);
    sincos(x[i], &s2, &c2);
    o[8 * i + 0] = s; o[8 * i + 1] = c; o[8 * i + 2] = s2; o[8 * i + 3] = c2;
    o[8 * i + 4] = fm_atan(x[i]); o[8 * i + 5] = atan(x[i]);
    o[8 * i + 6] = fm_atan2(y[i], x[i]); o[8 * i + 7] = atan2(y[i], x[i]);
}

static double ulp_err(double got, long double ref) {
    if (std::isnan(got) && std::isnan((double)ref)) return 0.0;
    if (std::isnan(got) != std::isnan((double)ref)) return 1e30;
    const double r = (double)ref;
    if (std::isinf(r) || std::isinf(got)) return got == r ? 0.0 : 1e30;
    const double u = std::nextafter(std::fabs(r), INFINITY) - std::fabs(r);
    return (double)(std::fabs((long double)got - ref) / (long double)(u > 0 ? u : 4.9e-324));
}

int main() {
    const int n = 1 << 22;
    std::mt19937_64 g(1);
    struct Range { const char* name; double lo, hi; };
    const Range rs[] = {{"[-pi/4, pi/4]", -0.785, 0.785}, {"[-4, 4]", -4, 4}, {"[-40, 40]", -40, 40},
                        {"[-1e5, 1e5]", -1e5, 1e5}, {"[-0.01, 0.01]", -0.01, 0.01}, {"[-1e3, 1e3]", -1e3, 1e3}};
    double *dx, *dy, *dout;
    (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&dy, n * 8); (void)hipMalloc(&dout, n * 64);
    std::vector<double> x(n), y(n), o(8 * (size_t)n);
    int bad = 0;
    for (const Range& R : rs) {
        std::uniform_real_distribution<double> ux(R.lo, R.hi), uy(-3.0, 3.0);
        for (int i = 0; i < n; ++i) { x[i] = ux(g); y[i] = uy(g); }
        (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
        (void)hipMemcpy(dy, y.data(), n * 8, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(eval, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, dout, n);
        (void)hipMemcpy(o.data(), dout, (size_t)n * 64, hipMemcpyDeviceToHost);
        double mx[8] = {0}, sm[8] = {0};
        for (int i = 0; i < n; ++i) {
            const long double xs = x[i], ys = y[i];
            const long double ref[8] = {sinl(xs), cosl(xs), sinl(xs), cosl(xs), atanl(xs), atanl(xs), atan2l(ys, xs),
                                        atan2l(ys, xs)};
            for (int k = 0; k < 8; ++k) {
                const double e = ulp_err(o[8 * (size_t)i + k], ref[k]);
                mx[k] = std::fmax(mx[k], e);
                sm[k] += e;
            }
        }
        printf("%-16s sin fm %.2f/%.3f lib %.2f/%.3f | cos fm %.2f/%.3f lib %.2f/%.3f | atan fm %.2f/%.3f lib %.2f/%.3f"
               " | atan2 fm %.2f/%.3f lib %.2f/%.3f  (max/mean ulp)\n", R.name, mx[0], sm[0] / n, mx[2], sm[2] / n,
               mx[1], sm[1] / n, mx[3], sm[3] / n, mx[4], sm[4] / n, mx[5], sm[5] / n, mx[6], sm[6] / n, mx[7], sm[7] / n);
        if (mx[0] > 1.5 || mx[1] > 1.5 || mx[4] > 2 || mx[6] > 2) bad = 1;
    }
    // special cases: zeros, infinities, NaN, huge arguments
    const double sp[][2] = {{0.0, 0.0}, {-0.0, 0.0}, {0.0, -0.0}, {-0.0, -0.0}, {1.0, 0.0}, {-1.0, 0.0}, {1.0, -0.0},
                            {0.0, 1.0}, {-0.0, -1.0}, {INFINITY, 1.0}, {1.0, INFINITY}, {INFINITY, INFINITY},
                            {-INFINITY, -INFINITY}, {NAN, 1.0}, {1.0, NAN}, {1e300, 1e-300}, {1e-300, 1e300},
                            {3e6, 2.0}, {-1e22, 1.0}, {0.3, -0.3}, {1e-310, 1.0}};
    const int ns = sizeof(sp) / sizeof(sp[0]);
    for (int i = 0; i < ns; ++i) { x[i] = sp[i][0]; y[i] = sp[i][1]; }
    (void)hipMemcpy(dx, x.data(), ns * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dy, y.data(), ns * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(eval, dim3(1), dim3(64), 0, 0, dx, dy, dout, ns);
    (void)hipMemcpy(o.data(), dout, ns * 64, hipMemcpyDeviceToHost);
    for (int i = 0; i < ns; ++i) {
        const double es = ulp_err(o[8 * i], sinl((long double)x[i])), ec = ulp_err(o[8 * i + 1], cosl((long double)x[i]));
        const double ea = ulp_err(o[8 * i + 4], atanl((long double)x[i]));
        const double e2 = ulp_err(o[8 * i + 6], atan2l((long double)y[i], (long double)x[i]));
        const bool sgn = std::signbit(o[8 * i + 6]) == std::signbit(o[8 * i + 7]) && std::signbit(o[8 * i + 4]) == std::signbit(o[8 * i + 5]);
        const bool ok = es <= 1.5 && ec <= 1.5 && ea <= 2 && e2 <= 2 && sgn;
        if (!ok) bad = 1;
        printf("special x=%g y=%g: sin %.2f cos %.2f atan %.2f atan2 %.2f (fm %.17g lib %.17g) %s\n", x[i], y[i], es, ec,
               ea, e2, o[8 * i + 6], o[8 * i + 7], ok ? "ok" : "BAD");
    }
    printf(bad ? "FASTMATH CHECK FAILED\n" : "FASTMATH CHECK OK\n");
    return bad;
}
