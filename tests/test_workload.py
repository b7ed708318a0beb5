"""Synthetic workloads (BASELINE.json configs): determinism and rank-independent sharding."""
import numpy as np

from trajectory_generation_amd.workload import SPLINE_KNOTS_X, make_workload, spline_eval
from trajectory_generation_amd.batch import spline_natural, vref_ramp


def test_shards_equal_slices_of_the_whole():
    whole = make_workload(16, 20, 0.05, kind="spline", seed=3)
    for r in range(4):
        part = make_workload(4, 20, 0.05, kind="spline", seed=3, id_offset=4 * r)
        np.testing.assert_array_equal(part["x0"], whole["x0"][4 * r:4 * r + 4])
        np.testing.assert_array_equal(part["ids"], np.arange(4 * r, 4 * r + 4))
        for a, b in zip(part["knots"], whole["knots"][4 * r:4 * r + 4]):
            np.testing.assert_array_equal(a[1], b[1])


def test_mixed_kinds_and_ranges():
    w = make_workload(64, 40, 0.05, kind="mixed", seed=1)
    assert set(w["kinds"].tolist()) == {0, 1}
    x0 = w["x0"]
    assert np.all((x0[:, 3] >= 0.4) & (x0[:, 3] <= 1.5)) and np.all(np.abs(x0[:, 4]) <= 0.05)
    np.testing.assert_allclose(w["vref"], vref_ramp(40, 0.05))


def test_spline_natural_and_eval(oracle_lib):
    rng = np.random.default_rng(0)
    yk = rng.uniform(-1, 1, len(SPLINE_KNOTS_X))
    coef = spline_natural(SPLINE_KNOTS_X, yk)
    np.testing.assert_allclose(coef.reshape(-1), oracle_lib.spline_natural(SPLINE_KNOTS_X, yk), atol=1e-12)
    # interpolates the knots, natural end conditions (second derivative 0 at both ends)
    for x, y in zip(SPLINE_KNOTS_X, yk):
        assert abs(spline_eval(SPLINE_KNOTS_X, coef, x)[0] - y) < 1e-12
    assert abs(coef[0, 2]) < 1e-14
    h = SPLINE_KNOTS_X[-1] - SPLINE_KNOTS_X[-2]
    assert abs(2 * coef[-1, 2] + 6 * coef[-1, 3] * h) < 1e-12
    try:
        from scipy.interpolate import CubicSpline
        cs = CubicSpline(SPLINE_KNOTS_X, yk, bc_type="natural")
        xs = np.linspace(SPLINE_KNOTS_X[0], SPLINE_KNOTS_X[-1], 97)
        np.testing.assert_allclose([spline_eval(SPLINE_KNOTS_X, coef, x)[0] for x in xs], cs(xs), atol=1e-12)
    except ImportError:
        pass
