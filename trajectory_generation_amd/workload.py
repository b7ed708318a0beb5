"""Synthetic closed-loop workloads (BASELINE.json configs).

The reference's only closed-loop caller is MPC/main.py:85-101 (one parabola, one trajectory).
These generators build B independent trajectories of the same loop with the geometry defined
in DESIGN.md "reference paths":
  * spline  (config 2 / 4): natural cubic spline y(x) through 11 knots x in [-6, 34] m (4 m
    spacing), y ~ U(-1, 1) m; linear extrapolation outside the knots.  Deviation from SURVEY.md
    8(d) config 2 (6 knots on x in [0, 12]), deliberate: a trajectory starts at X in [-2, 2] and,
    on the 0.8 -> 2.0 m/s ramp, covers about 17 m in the bench's 205 steps and 22 m in the dataset's
    240 -- with knots on [0, 12] only, it would start on the extrapolated line and spend most of the
    run past the last knot tracking a straight line (trivially easy QPs); the 4 m spacing keeps the
    curvature of 6 knots over 12 m (2.4 m spacing) within a factor of 2.
  * mixed   (config 3): 50 % sinusoid y = A sin(w x + phase) (A = 0.5, w = 0.5 of MPC/README.md:75,
    jittered +-20 %), 50 % parabola y = a x^2 (a = 0.1 of main.py:64-66, drawn in [0.05, 0.15]).
Initial state per trajectory (ranges of generation_type1.py:260-265 / main.py:77): X ~ U(-2, 2),
Y = y(X) + U(-0.5, 0.5), phi = atan(y'(X)) + U(-0.2, 0.2), vx ~ U(0.4, 1.5), vy ~ U(-0.05, 0.05),
omega ~ U(-1, 1); u_prev = [d_ss(vx), 0] (main.py:20-22).  vref = the main.py:28-32 ramp
(0.8 -> 2.0 m/s over 2 s) over the horizon, re-used every step (main.py:87).
Trajectory `tid` draws from numpy.random.default_rng([seed, tid]) so shards are reproducible
for any rank count.
"""
from __future__ import annotations

import numpy as np

from .batch import d_steady_state, spline_natural, vref_ramp

SPLINE_KNOTS_X = np.linspace(-6.0, 34.0, 11)


def spline_eval(xk, coef, x):
    """y, dy/dx of the natural spline (same rule as the kernel's path_eval)."""
    nk = len(xk)
    if x <= xk[0]:
        return coef[0, 0] + coef[0, 1] * (x - xk[0]), coef[0, 1]
    if x >= xk[-1]:
        q = coef[nk - 2]
        h = xk[-1] - xk[-2]
        ye = q[0] + h * (q[1] + h * (q[2] + h * q[3]))
        se = q[1] + h * (2 * q[2] + h * 3 * q[3])
        return ye + se * (x - xk[-1]), se
    j = min(int(np.searchsorted(xk, x, side="right")) - 1, nk - 2)
    q = coef[j]
    t = x - xk[j]
    return q[0] + t * (q[1] + t * (q[2] + t * q[3])), q[1] + t * (2 * q[2] + t * 3 * q[3])


def _initial_state(rng, y, dy):
    X = rng.uniform(-2.0, 2.0)
    yy, dd = y(X), dy(X)
    return np.array([X, yy + rng.uniform(-0.5, 0.5), np.arctan(dd) + rng.uniform(-0.2, 0.2),
                     rng.uniform(0.4, 1.5), rng.uniform(-0.05, 0.05), rng.uniform(-1.0, 1.0)])


def make_workload(B, N=20, Ts=0.05, kind="spline", seed=0, id_offset=0):
    """Returns dict(kinds [B], pcs [B,4], knots list, x0 [B,6], u0 [B,2], vref [N+1], ids [B])."""
    kinds, pcs, knots, x0 = [], [], [], []
    for i in range(B):
        tid = id_offset + i
        rng = np.random.default_rng([seed, tid])
        if kind == "spline":
            yk = rng.uniform(-1.0, 1.0, len(SPLINE_KNOTS_X))
            coef = spline_natural(SPLINE_KNOTS_X, yk)
            x0.append(_initial_state(rng, lambda x: spline_eval(SPLINE_KNOTS_X, coef, x)[0],
                                     lambda x: spline_eval(SPLINE_KNOTS_X, coef, x)[1]))
            kinds.append(2); pcs.append([0.0] * 4); knots.append((SPLINE_KNOTS_X.copy(), yk))
        elif kind == "mixed":
            if tid % 2 == 0:
                A = 0.5 * rng.uniform(0.8, 1.2); w = 0.5 * rng.uniform(0.8, 1.2); ph = rng.uniform(0, 2 * np.pi)
                c = [A, w, ph, 0.0]
                x0.append(_initial_state(rng, lambda x: A * np.sin(w * x + ph), lambda x: A * w * np.cos(w * x + ph)))
                kinds.append(1)
            else:
                a = rng.uniform(0.05, 0.15)
                c = [0.0, 0.0, a, 0.0]
                x0.append(_initial_state(rng, lambda x: a * x * x, lambda x: 2 * a * x))
                kinds.append(0)
            pcs.append(c); knots.append(None)
        elif kind == "parabola":
            a = 0.1
            x0.append(np.array([0.0, 0.5, 0.0, 1.0, 0.0, 0.0]))   # main.py:77
            kinds.append(0); pcs.append([0.0, 0.0, a, 0.0]); knots.append(None)
        else:
            raise ValueError(kind)
    x0 = np.array(x0)
    u0 = np.stack([np.array([d_steady_state(v), 0.0]) for v in x0[:, 3]])
    return dict(kinds=np.array(kinds, np.int32), pcs=np.array(pcs, np.float64), knots=knots, x0=x0, u0=u0,
                vref=vref_ramp(N, Ts), ids=np.arange(id_offset, id_offset + B))

