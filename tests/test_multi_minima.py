"""Evidence for the one multi-minimum parity case.

`tests/test_gpu_ipm.py` MULTI_MINIMA: one_room_switch at the tight options (bilinear dynamics, a
switched objective) has several local minima, and which one an interior-point run reaches is
decided by rounding.  Here the ORACLE alone shows it (CPU, no kernel involved): the same NLP,
started from w0 and from w0 moved by a seeded relative 1e-12 perturbation, converges
(Solve_Succeeded, tol 1e-10) to two different local minima, 1.8 apart in the objective, after
different iteration counts.  A kernel run, whose arithmetic differs from the oracle's by more than
1e-12 from the first iteration on, is therefore checked there for reaching a local minimum of the
NLP (the oracle warm-started at its point converges in place), not for reaching the oracle's.
`scripts/multi_minima.py` runs the wider scan recorded in profiles/r06/multi_minima.txt.
"""

import numpy as np

from oracle import ipm
from tests import configs

TIGHT = ipm.IPMOptions(tol=1e-10, max_iter=500, acceptable_iter=0)


def perturbed(w0, seed: int, k: int, rel: float = 1e-12):
    """The k-th seeded relative perturbation of w0 (the scan's draws, in order)."""
    rng = np.random.default_rng(seed)
    for _ in range(k):
        rng.standard_normal(w0.shape)
    return w0 * (1.0 + rel * rng.standard_normal(w0.shape))


def test_oracle_reaches_different_minima_from_1e12_perturbations():
    case = configs.CASES["one_room_switch"]()
    p, lbw, ubw, w0 = case.oracle_inputs
    fns, lbg, ubg = case.oracle.functions(p), case.oracle.lbg(p), case.oracle.ubg(p)
    a = ipm.solve(fns, w0, lbw, ubw, lbg, ubg, TIGHT)
    w1 = perturbed(w0, seed=0, k=1)
    assert np.max(np.abs(w1 - w0) / np.maximum(np.abs(w0), 1e-300)) < 1e-11
    b = ipm.solve(fns, w1, lbw, ubw, lbg, ubg, TIGHT)
    assert a.success and b.success, (a.status, b.status)
    # two local minima of the same NLP, far apart at the parity tolerance (rel 1e-6)
    assert abs(a.f - 5714.008148) < 1e-3 and abs(b.f - 5715.828115) < 1e-3, (a.f, b.f)
    assert abs(a.f - b.f) / abs(a.f) > 1e-4
    assert a.iterations != b.iterations
    # each is a minimum: the oracle warm-started at it stays there
    warm = ipm.IPMOptions(tol=1e-10, max_iter=50, acceptable_iter=0, mu_init=1e-9, bound_push=1e-9, bound_frac=1e-9)
    for r in (a, b):
        c = ipm.solve(fns, r.x, lbw, ubw, lbg, ubg, warm)
        assert c.success and c.iterations <= 10, (c.status, c.iterations)
        np.testing.assert_allclose(c.f, r.f, rtol=1e-9)
