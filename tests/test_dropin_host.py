"""Host side of the drop-in mpc_step (no GPU): the per-call struct cache returns the struct built for the same
arguments (exact keys: arrays by bytes) and a fresh one for any argument that differs."""
import numpy as np

from trajectory_generation_amd import batch as TB, mpc_6stati as M


def _cfg(**kw):
    args = dict(N=20, Ts=0.05, q_c=6.0, q_phi=0.5, q_vx=0.5, R=np.diag([0.02, 2.0]), Rd=np.diag([0.01, 5.0]),
                u_bounds=((-1.0, 1.0), (-0.6, 0.6)), du_bounds=((-0.5, 0.5), (-0.3, 0.3)), x_lo=None, x_hi=None)
    args.update(kw)
    key = [args[k] for k in ("N", "Ts", "q_c", "q_phi", "q_vx", "R", "Rd", "u_bounds", "du_bounds", "x_lo", "x_hi")]
    return M._cached_struct("cfg", lambda: TB.config_struct(**args), *key, ())


def test_struct_cache_same_arguments_same_struct():
    a, b = _cfg(), _cfg()
    assert a is b
    assert bytes(a) == bytes(TB.config_struct(N=20, Ts=0.05))


def test_struct_cache_distinguishes_every_argument():
    base = _cfg()
    for kw in (dict(N=21), dict(Ts=0.02), dict(q_c=6.5), dict(R=np.diag([0.02, 2.5])), dict(Rd=np.diag([0.02, 5.0])),
               dict(u_bounds=((-1.0, 1.0), (-0.5, 0.6))), dict(x_lo=np.full(6, -1e3)), dict(x_hi=np.full(6, 1e3))):
        c = _cfg(**kw)
        assert c is not base and bytes(c) != bytes(base), kw
        assert bytes(c) == bytes(TB.config_struct(**{**dict(N=20, Ts=0.05), **kw})), kw


def test_struct_cache_unhashable_builds_fresh():
    built = []
    s1 = M._cached_struct("cfg", lambda: built.append(1) or TB.config_struct(), object())
    s2 = M._cached_struct("cfg", lambda: built.append(1) or TB.config_struct(), object())
    assert len(built) == 2 and s1 is not s2


def test_struct_cache_keys_signed_zeros_and_types_apart():
    """-0.0 and 0.0 (and 1, 1.0, True) are distinct keys: a cached struct is exactly what config_struct builds for the
    arguments given (a -0.0 bound is kept as -0.0, which the clamp's sign of zero follows)."""
    keys = [M._frozen(v) for v in (0.0, -0.0, 1, 1.0, True, np.float32(0.0))]
    assert len(set(keys)) == 6
    assert M._frozen(np.float64(-0.0)) == M._frozen(-0.0)   # (a float64 scalar is the same double)
    a = _cfg(u_bounds=((-1.0, 1.0), (-0.6, 0.0)))
    b = _cfg(u_bounds=((-1.0, 1.0), (-0.6, -0.0)))
    assert a is not b
    assert bytes(b) == bytes(TB.config_struct(N=20, Ts=0.05, u_bounds=((-1.0, 1.0), (-0.6, -0.0))))


def test_params_key_exact_and_fast_path():
    """The drop-in's params key (_params_key: names + the values' bits in one pack) separates every changed value,
    signed zeros included, and leaves non-float values to the generic key (None); the cached params struct is the
    one params_struct builds."""
    p = dict(M.Params)
    k0 = M._params_key(p)
    assert k0 is not None and k0 == M._params_key(dict(M.Params))
    for name in p:
        q = dict(p)
        q[name] = p[name] * (1.0 + 1e-12) if p[name] != 0.0 else 1e-300
        assert M._params_key(q) != k0, name
    z0, z1 = dict(p, vx_zero=0.0), dict(p, vx_zero=-0.0)
    assert M._params_key(z0) != M._params_key(z1)
    assert M._params_key(dict(p, m=1)) is None and M._params_key(dict(p, m=np.float64(0.041))) is None
    s = M._cached_struct("params", lambda: TB.params_struct(p), key=k0)
    assert s is M._cached_struct("params", lambda: TB.params_struct(p), key=M._params_key(dict(M.Params)))
    assert bytes(s) == bytes(TB.params_struct(p))
