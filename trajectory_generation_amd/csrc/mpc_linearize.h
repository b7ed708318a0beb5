// mpc_linearize.h -- kernel 1 of the MPC step: nominal rollout + central-difference linearization.
//
// Reference: MPC/mpc_6stati.py:165-178 (rollout and the N linearization points), :73-97
// (numerical_jacobian, eps = 1e-5), :99-109 (A = I + Ts Jx, B = Ts Ju, g = x + Ts f - A x - B u).
// One 64-lane wave per instance.  Lane 0 runs the (serial) Euler rollout; the 6 non-trivial
// Jacobian columns of every stage (phi, vx, vy, omega, d, delta) are then independent items, one
// lane each, 2 f_cont evaluations per item.  Columns X and Y are exactly zero (f does not read
// X, Y, so the reference's f(x+dx) - f(x-dx) is 0.0 bit for bit) and are not evaluated.
// A, B, g are staged in LDS and written to the workspace as [B,N,36], [B,N,12], [B,N,6] float64,
// where the solve kernel (mpc_solve.h) reads them back (L2 / Infinity-Cache resident).
#pragma once
#include "mpc_common.h"

namespace tgmpc {

template <int NM, bool CLOSED>
__global__ __launch_bounds__(64) void linearize_kernel(const KArgs a) {
    __shared__ double s_xbar[(NM + 1) * 6];
    __shared__ double s_fbar[NM * 6];
    __shared__ double s_A[NM * 36];
    __shared__ double s_B[NM * 12];
    __shared__ double s_g[NM * 6];
    __shared__ double s_x0[6], s_up[2];

    const traj_vehicle_params& p = a.p;
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    const int N = a.c.N;
    const double Ts = a.c.Ts;

    if (CLOSED) {
        if (t < 6) s_x0[t] = a.x_state[6 * b + t];
        if (t < 2) s_up[t] = a.u_state[2 * b + t];
    } else {
        if (t < 6) s_x0[t] = a.x0[6 * b + t];
        if (t < 2) s_up[t] = a.u_prev[2 * b + t];
    }
    __syncthreads();

    // nominal rollout (:165-172), constant input u_prev
    if (t == 0) {
        double x[6], f[6], sd, cd;
        sincos(s_up[1], &sd, &cd);
        for (int i = 0; i < 6; ++i) {
            x[i] = s_x0[i];
            s_xbar[i] = x[i];
        }
        for (int k = 0; k < N; ++k) {
            f_cont_sc(p, x, s_up[0], s_up[1], sd, cd, f);
            for (int i = 0; i < 6; ++i) {
                s_fbar[6 * k + i] = f[i];
                x[i] = x[i] + Ts * f[i];
                s_xbar[6 * (k + 1) + i] = x[i];
            }
        }
    }
    __syncthreads();

    // Jacobian columns (:73-97): item = (stage k, column col), col 0..5 states, 6..7 inputs
    const double eps = 1e-5;
    for (int it = t; it < 8 * N; it += 64) {
        const int k = it >> 3, col = it & 7;
        double J[6] = {0, 0, 0, 0, 0, 0};
        if (col >= 2) {
            double xp[6], xm[6], up[2], um[2], fp[6], fm[6];
            // exactly the reference's vectors: the perturbed argument is x + dx / x - dx with
            // dx = eps e_col (so x_i + 0.0 elsewhere), the other argument is passed unchanged
            const bool on_x = col < 6;
            for (int i = 0; i < 6; ++i) {
                const double xi = s_xbar[6 * k + i], d = (i == col) ? eps : 0.0;
                xp[i] = on_x ? xi + d : xi;
                xm[i] = on_x ? xi - d : xi;
            }
            for (int i = 0; i < 2; ++i) {
                const double ui = s_up[i], d = (i + 6 == col) ? eps : 0.0;
                up[i] = on_x ? ui : ui + d;
                um[i] = on_x ? ui : ui - d;
            }
            f_cont(p, xp, up, fp);
            f_cont(p, xm, um, fm);
            for (int r = 0; r < 6; ++r) J[r] = (fp[r] - fm[r]) / (2.0 * eps);
        }
        // :106-107  Ad = I + Ts Jx ; Bd = Ts Ju
        for (int r = 0; r < 6; ++r) {
            if (col < 6) s_A[k * 36 + r * 6 + col] = ((r == col) ? 1.0 : 0.0) + Ts * J[r];
            else s_B[k * 12 + r * 2 + (col - 6)] = Ts * J[r];
        }
    }
    __syncthreads();
    // :108  g = x_bar + Ts f - Ad x_bar - Bd u_bar   (f = the rollout's f(x_bar_k, u_prev))
    for (int it = t; it < 6 * N; it += 64) {
        const int k = it / 6, r = it % 6;
        double ax = 0.0, bu = 0.0;
        for (int cc = 0; cc < 6; ++cc) ax += s_A[k * 36 + r * 6 + cc] * s_xbar[6 * k + cc];
        for (int cc = 0; cc < 2; ++cc) bu += s_B[k * 12 + r * 2 + cc] * s_up[cc];
        s_g[6 * k + r] = s_xbar[6 * k + r] + Ts * s_fbar[6 * k + r] - ax - bu;
    }
    __syncthreads();
    // coalesced write-out
    const size_t o = (size_t)b * N;
    for (int i = t; i < 36 * N; i += 64) a.wsA[o * 36 + i] = s_A[i];
    for (int i = t; i < 12 * N; i += 64) a.wsB[o * 12 + i] = s_B[i];
    for (int i = t; i < 6 * N; i += 64) a.wsg[o * 6 + i] = s_g[i];
}

}  // namespace tgmpc
