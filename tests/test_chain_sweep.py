"""The state-chain pivot blocks are inverted by a Bunch-Kaufman-pivoted symmetric sweep
(csrc/mpcx_ipm.hip ``bk_sweep``); this is its host restatement, checked against numpy on
random symmetric indefinite blocks of the chain sizes (RNGRoom 4x4, MHE 6x6, NARX 7x7),
including saddle blocks with a zero leading part (the bordered multipliers): the inverse
and the inertia (which the inertia correction reads) must match.  The GPU parity cases of
those models (tests/test_gpu_ipm.py, tests/test_gpu_admm.py) run the kernel itself."""

import numpy as np
import pytest

ALPHA = (1 + 17 ** 0.5) / 8   # BK_ALPHA
ZERO_PIVOT = 1e-20


def sweep(A0):
    """Line by line the kernel's loop: first unswept index k, BK pivot choice among the
    unswept indices, one read-modify-write of the whole block per pivot."""
    A = np.array(A0, float)
    n = len(A)
    done = np.zeros(n, bool)
    zero = np.zeros(n, bool)
    pos = neg = nz = 0
    while not done.all():
        k = int(np.argmin(done))
        cand = [i for i in range(n) if not done[i] and i != k]
        r = max(cand, key=lambda i: (abs(A[i, k]), -i)) if cand else -1
        lam = abs(A[r, k]) if cand else 0.0
        akk = abs(A[k, k])
        p, q = k, -1
        if not (max(akk, lam) == 0.0 or akk >= ALPHA * lam):
            sigma = max(abs(A[r, j]) for j in range(n) if not done[j] and j != r)
            if akk * sigma >= ALPHA * lam * lam:
                p = k
            elif abs(A[r, r]) >= ALPHA * sigma:
                p = r
            else:
                q = r
        B = A.copy()
        if q < 0:
            d = A[p, p]
            done[p] = True
            if abs(d) <= ZERO_PIVOT:
                nz += 1
                zero[p] = True
                continue
            pos, neg = (pos + 1, neg) if d > 0 else (pos, neg + 1)
            B[:, :] = A - np.outer(A[:, p], A[p, :]) / d
            B[p, :] = A[p, :] / d
            B[:, p] = A[:, p] / d
            B[p, p] = -1.0 / d
        else:
            P = [k, q]
            Pb = A[np.ix_(P, P)]
            det = Pb[0, 0] * Pb[1, 1] - Pb[0, 1] ** 2
            done[P] = True
            if abs(det) <= ZERO_PIVOT ** 2:
                nz += 2
                zero[P] = True
                continue
            if det < 0:
                pos, neg = pos + 1, neg + 1
            elif Pb[0, 0] + Pb[1, 1] > 0:
                pos += 2
            else:
                neg += 2
            Pi = np.array([[Pb[1, 1], -Pb[0, 1]], [-Pb[0, 1], Pb[0, 0]]]) / det
            B[:, :] = A - A[:, P] @ Pi @ A[P, :]
            B[P, :] = Pi @ A[P, :]
            B[:, P] = A[:, P] @ Pi
            B[np.ix_(P, P)] = -Pi
        A = B
    out = -A
    out[zero, :] = 0.0
    out[:, zero] = 0.0
    return out, (pos, neg, nz)


@pytest.mark.parametrize("n", [4, 6, 7])
def test_sweep_inverse_and_inertia(n):
    rng = np.random.default_rng(n)
    for t in range(300):
        M = rng.normal(size=(n, n))
        M = M + M.T
        if t % 3 == 0:            # bordered multipliers: zero leading block
            M[:n // 2, :n // 2] = 0.0
        if t % 5 == 0:            # barrier-scaled diagonal
            M[np.diag_indices(n)] *= 10.0 ** rng.integers(-6, 7, n)
        inv, (pos, neg, nz) = sweep(M)
        ev = np.linalg.eigvalsh(M)
        assert (pos, neg, nz) == ((ev > 0).sum(), (ev < 0).sum(), 0)
        ref = np.linalg.inv(M)
        np.testing.assert_allclose(inv, ref, rtol=1e-7, atol=1e-7 * np.abs(ref).max())


def test_sweep_reports_zero_pivot():
    M = np.diag([2.0, 0.0, -1.0])
    inv, (pos, neg, nz) = sweep(M)
    assert (pos, neg, nz) == (1, 1, 1)
    np.testing.assert_array_equal(inv, np.diag([0.5, 0.0, -1.0]))
