"""The row-split kernel's block sweep (csrc/mpc_split.h, TGMPC_SPLIT_BLOCK), restated per row in numpy: for a block P of
m pivots every row forms the block's LDL' in the sequential sweep's elimination order and its coefficient vector
w = D^-1 z (z = -K[r][P] outside the block, e_k on the block's k-th pivot row), then row r <- base + sum_k w_k K[.][p+k]
(base = row r, or an exact zero row on the pivot rows; the pivot rows' entries are the published column values) and
K[r][P] <- -w.  After all blocks the matrix is -K^-1 (the kernel negates it).  CPU-only: the algebra, not the kernel
(the GPU parity suite checks the kernel's results against the oracle)."""
import numpy as np
import pytest


def block_sweep(K, m, n_real=None):
    K = K.copy()
    n = K.shape[0]
    n_real = n if n_real is None else n_real
    for p in range(0, n, m):
        if p >= n_real:
            continue   # a padding block: identity rows, nothing to eliminate
        P = list(range(p, p + m))
        Dl = np.zeros((m, m))
        for k in range(m):
            for i in range(k, m):
                Dl[i, k] = K[p + i, p + k]
        dinv = np.zeros(m)
        L = np.zeros((m, m))
        for k in range(m):
            assert Dl[k, k] > 0
            dinv[k] = 1.0 / Dl[k, k]
            for i in range(k + 1, m):
                L[i, k] = Dl[i, k] * dinv[k]
                for j in range(k + 1, i + 1):
                    Dl[i, j] = -L[i, k] * Dl[j, k] + Dl[i, j]
        cols = K[:, P].copy()
        new = np.zeros_like(K)
        for r in range(n):
            kp = r - p
            inb = 0 <= kp < m
            w = np.array([(1.0 if i == kp else 0.0) if inb else -K[r, p + i] for i in range(m)])
            for k in range(m):
                for i in range(k + 1, m):
                    w[i] = -L[i, k] * w[k] + w[i]
            w = w * dinv
            for k in range(m - 1, -1, -1):
                for i in range(k + 1, m):
                    w[k] = -L[i, k] * w[i] + w[k]
            row = (np.zeros(n) if inb else K[r].copy()) + cols @ w
            row[P] = -w
            new[r] = row
        K = new
    return -K


@pytest.mark.parametrize("n,m", [(8, 1), (8, 2), (8, 4), (40, 2), (40, 4), (80, 4)])
def test_block_sweep_is_the_inverse(n, m):
    rng = np.random.default_rng(n + m)
    A = rng.standard_normal((n, n))
    K = A @ A.T + n * np.eye(n)
    inv = np.linalg.inv(K)
    assert np.abs(block_sweep(K, m) - inv).max() <= 1e-13 * np.abs(inv).max()


@pytest.mark.parametrize("m", [2, 4])
def test_block_sweep_with_identity_padding(m):
    """n = 2N real variables padded to a multiple of the block with identity rows (as the kernel pads to 2H): the
    real block of the result is the real problem's inverse, whether a block is all padding or straddles n."""
    rng = np.random.default_rng(7)
    n_real, n = 78, 80
    A = rng.standard_normal((n_real, n_real))
    Kr = A @ A.T + n_real * np.eye(n_real)
    K = np.eye(n)
    K[:n_real, :n_real] = Kr
    R = block_sweep(K, m, n_real=n_real if m == 2 else n)   # m = 4: the last block straddles n (identity pivots)
    inv = np.linalg.inv(Kr)
    assert np.abs(R[:n_real, :n_real] - inv).max() <= 1e-13 * np.abs(inv).max()
