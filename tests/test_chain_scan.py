"""Host restatement of the scalar state chain's scan (csrc/mpcx_ipm.hip chain_factor, NX = 1,
no bordered rows): the pivots d_j = a_j - b_j / d_{j-1} as ratios of the leading minors
p_j = a_j p_{j-1} - b_j p_{j-2}, the prefix products of M_j = [[a_j, -b_j], [1, 0]] formed by a
Hillis-Steele scan with each partial product rescaled by a power of two.  Checked against the
serial recurrence (what the kernel falls back to near a zero pivot) and the eigenvalue inertia
of the tridiagonal matrix."""

import math

import numpy as np
import pytest


def serial(a, b):
    d, dprev = np.zeros(len(a)), 0.0
    for j in range(len(a)):
        d[j] = a[j] - b[j] * dprev
        dprev = 1.0 / d[j]
    return d


def scan(a, b):
    """The kernel's scan, lane j = entry j (N <= 16: one DPP row)."""
    n = len(a)
    P = [np.array([[a[j], -b[j]], [1.0, 0.0]]) for j in range(n)]
    sh = 1
    while sh < n:
        Q = [p.copy() for p in P]
        for j in range(sh, n):
            r = P[j] @ Q[j - sh]
            mx = np.abs(r).max()
            e = math.frexp(mx)[1] - 1 if 0.0 < mx < np.inf else 0   # ilogb
            P[j] = np.ldexp(r, -e)
        sh <<= 1
    return np.array([p[0, 0] / p[1, 0] for p in P])


def tridiag(a, b):
    """The chain matrix: diagonal a, off-diagonal sqrt(b) (b_j = s_j^2)."""
    n = len(a)
    T = np.diag(a)
    for j in range(1, n):
        T[j, j - 1] = T[j - 1, j] = math.sqrt(b[j])
    return T


@pytest.mark.parametrize("seed", range(20))
@pytest.mark.parametrize("n", [1, 2, 7, 15, 16])
def test_scan_matches_serial_recurrence_and_inertia(seed, n):
    rng = np.random.default_rng(seed)
    scale = 10.0 ** rng.uniform(-6, 8, n)          # barrier terms span many decades
    b = np.concatenate([[0.0], rng.uniform(0.0, 1.0, n - 1) * scale[1:] * scale[:-1]])
    a = scale * rng.uniform(1.05, 3.0, n) + np.concatenate([[0.0], np.sqrt(b[1:])])
    if seed % 4 == 3:                                # indefinite chains (inertia correction)
        a[rng.integers(0, n)] *= -1.0
    ds, dq = serial(a, b), scan(a, b)
    ok = np.all(np.isfinite(dq)) and np.all(np.abs(dq) > 1e-8 * np.abs(a))
    if not ok:
        pytest.skip("the kernel takes the serial recurrence for this chain")
    np.testing.assert_allclose(dq, ds, rtol=1e-9)
    ev = np.linalg.eigvalsh(tridiag(a, b))
    assert int((dq > 0).sum()) == int((ev > 0).sum())


def test_scan_survives_the_range_of_a_restoration_chain():
    """Products of 15 pivots of ~1e20 (restoration penalties) overflow without the rescaling."""
    n = 15
    a = np.full(n, 3e20)
    b = np.concatenate([[0.0], np.full(n - 1, 1e40)])
    np.testing.assert_allclose(scan(a, b), serial(a, b), rtol=1e-12)


def accepted(a, b, d):
    """The kernel's acceptance of a scanned chain (else it runs the serial recurrence): finite
    pivots away from zero relative to their diagonals, each satisfying the recurrence with its
    neighbour's pivot to the rounding of its terms."""
    r = 1.0 / d
    rprev = np.concatenate([[0.0], r[:-1]])
    rec = a - b * rprev
    return bool(np.all(np.isfinite(d)) and np.all(np.abs(d) > 1e-8 * np.abs(a)) and np.all(np.abs(d) > 1e-20)
                and np.all(np.abs(d - rec) <= 1e-12 * (np.abs(a) + np.abs(b * rprev))))


@pytest.mark.parametrize("seed", range(40))
def test_accepted_scans_agree_with_the_recurrence_on_near_singular_chains(seed):
    """Chains with strong cancellation (each pivot 1e-3..1e-7 of its diagonal, indefinite signs: the
    restoration phase's chains): whenever the kernel's checks accept the scan, its pivots agree with
    the serial recurrence; rejected chains take the recurrence itself."""
    rng = np.random.default_rng(100 + seed)
    n = 15
    a = 10.0 ** rng.uniform(-2, 6, n) * rng.choice([-1.0, 1.0], n)
    b = np.zeros(n)
    d = np.zeros(n)
    d[0] = a[0]
    for j in range(1, n):   # b_j chosen so that d_j = a_j - b_j / d_{j-1} is a tiny fraction of a_j
        target = a[j] * 10.0 ** rng.uniform(-7, -3)
        b[j] = abs((a[j] - target) * d[j - 1])
        d[j] = a[j] - b[j] / d[j - 1]
    ds, dq = serial(a, b), scan(a, b)
    if accepted(a, b, dq):
        np.testing.assert_allclose(dq, ds, rtol=1e-6)
