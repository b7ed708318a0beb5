"""The arithmetic of knet_fc2x_kernel (csrc/knet.hip) restated in numpy: a float32 value split into three bf16
terms (each rounded to nearest even, the residuals formed in float32) is represented exactly, and the six kept
term products of a b differ from the exact product by less than 2^-23 |a b|, the size of one float32 rounding of
the product.  CPU only; the GPU kernel itself is checked against float64 in tests/test_knet_fc2.py."""
import numpy as np


def _bf16(x):
    b = x.astype(np.float32).view(np.uint32).astype(np.uint64)
    b = (b + 0x7FFF + ((b >> 16) & 1)) >> 16 << 16          # round to nearest even at bit 16
    return b.astype(np.uint32).view(np.float32)


def _split(v):
    h = _bf16(v)
    r1 = (v - h).astype(np.float32)
    m = _bf16(r1)
    r2 = (r1 - m).astype(np.float32)
    return h, m, _bf16(r2), r2


def test_three_term_split_is_exact():
    rng = np.random.default_rng(0)
    x = (rng.normal(size=200_000) * np.exp(rng.normal(size=200_000) * 6)).astype(np.float32)
    h, m, lo, r2 = _split(x)
    assert np.array_equal(lo, r2)                            # the last residual is already a bf16
    assert np.array_equal(h.astype(np.float64) + m + lo, x.astype(np.float64))


def test_six_products_within_one_f32_rounding():
    rng = np.random.default_rng(1)
    a = (rng.normal(size=200_000) * np.exp(rng.normal(size=200_000) * 3)).astype(np.float32)
    b = (rng.normal(size=200_000) * np.exp(rng.normal(size=200_000) * 3)).astype(np.float32)
    ah, am, al, _ = (t.astype(np.float64) for t in _split(a))
    bh, bm, bl, _ = (t.astype(np.float64) for t in _split(b))
    for p, q in ((ah, bh), (ah, bm), (am, bh), (ah, bl), (al, bh), (am, bm)):
        assert np.array_equal((p * q).astype(np.float32).astype(np.float64), p * q)   # exact in f32
    p6 = ah * bh + ah * bm + am * bh + ah * bl + al * bh + am * bm
    exact = a.astype(np.float64) * b.astype(np.float64)
    assert (np.abs(p6 - exact) <= 2.0 ** -23 * np.abs(exact)).all()
