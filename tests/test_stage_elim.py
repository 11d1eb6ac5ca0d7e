"""Generated static sparse elimination of the stage interiors (runtime/stage_elim.py).

The straight-line ``gen_stage_elim`` body of each benchmark structure is executed on
the host (runtime/elim_sim.py) on random KKT-shaped local systems with the model's
structure, and checked against dense numpy: interior inertia (Sylvester: pivot order
cannot change it), the back-substitution operators ``W = A_II^{-1} [A_IT | r_I]`` and
the Schur blocks / eliminated rhs the state chain receives.  The kernel runs the same
code (csrc/mpcx_ipm.hip ``static_stage``), so GPU parity then rests on the same body.
"""

import numpy as np
import pytest

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.runtime import elim_sim

MODELS = {
    "one_room": lambda: bm.one_room(),
    "one_room_radau3": lambda: bm.one_room(d=3, method="radau"),
    "one_room_du": lambda: bm.one_room(r_delta_mDot=0.1),
    "admm_room": lambda: bm.admm_room(),
    "admm_ahu": lambda: bm.admm_ahu(),
    "exchange_room": lambda: bm.exchange_room(),
    "exchange_supply": lambda: bm.exchange_supply(),
    "room_nn": lambda: bm.room_nn(),
    "tz_cca": lambda: bm.tz_cca(),
    "mhe_room": lambda: bm.mhe_room(),
    "rng_room_mpc": lambda: bm.rng_room_mpc(),
}


def _dims(gen):
    d = gen.dims
    nmu = len(gen.bordered_rows)
    ni = d["NV"] + d["NG"] - nmu
    nx, nc = d["NX"], d["NX"] + nmu
    return ni, d["NV"], nx, nc


def _random_system(gen, rng, plan=None):
    """Symmetric local system on the generated structure with KKT signs: primal
    diagonal > 0, paired (equality) dual diagonal 0, other dual diagonals < 0."""
    ni, nv, nx, nc = _dims(gen)
    P = np.array(gen.pattern, bool)
    n = P.shape[0]
    A = np.where(P, rng.uniform(-1.0, 1.0, (n, n)), 0.0)
    A = np.tril(A) + np.tril(A, -1).T
    paired = {i for b in (plan or gen.elim).blocks if len(b) == 2 for i in b}
    for i in range(n):
        if i < nv or i >= ni:
            A[i, i] = rng.uniform(0.5, 5.0) + np.abs(A[i]).sum()
        else:
            A[i, i] = 0.0 if i in paired else -rng.uniform(0.1, 2.0)
    return A


CASES = sorted(MODELS) + ["mhe_room:stage0"]


@pytest.mark.parametrize("name", CASES)
def test_generated_elimination_matches_dense(name):
    """``name:stage0``: the stage-0 plan (rows open at k = 0 pivot as inequalities)."""
    model, _, which = name.partition(":")
    be, _ = MODELS[model]()
    gen = be.problem.gen
    ni, nv, nx, nc = _dims(gen)
    ntr = nx + nc + 1
    plan, lines = (gen.elim0, gen.elim0_lines) if which else (gen.elim, gen.elim_lines)
    assert plan is not None
    code = elim_sim.compile_body(lines)
    rng = np.random.default_rng(11)
    for _ in range(5):
        A = _random_system(gen, rng, plan)
        out = elim_sim.run(code, elim_sim.compact(A, gen.compact), ni, ntr, nx * nx + nc * nc + nc * nx, nx + nc)
        assert not out["bad"]
        AII, AIT = A[:ni, :ni], A[:ni, ni:]
        ev = np.linalg.eigvalsh(AII)
        assert (out["pos"], out["neg"]) == (int((ev > 0).sum()), int((ev < 0).sum()))
        W = np.linalg.solve(AII, AIT)
        np.testing.assert_allclose(out["TR"].reshape(ntr, ni).T, W, rtol=1e-9, atol=1e-9 * np.abs(W).max())
        S = A[ni:, ni:] - AIT.T @ W
        want = np.concatenate([S[:nx, :nx].ravel(), S[nx:nx + nc, nx:nx + nc].ravel(), S[nx:nx + nc, :nx].ravel()])
        if want.size:
            np.testing.assert_allclose(out["S"][:want.size], want, rtol=1e-9, atol=1e-9 * np.abs(want).max())
        if nx + nc:
            np.testing.assert_allclose(out["ZX"][:nx + nc], S[-1, :nx + nc], rtol=1e-9,
                                       atol=1e-9 * max(1.0, np.abs(S[-1]).max()))


@pytest.mark.parametrize("name", ["one_room", "room_nn"])
def test_singular_static_pivot_is_reported_before_outputs(name):
    """A vanishing paired Jacobian entry (e.g. a fixed variable in a pair) makes a static
    2x2 pivot singular: the body reports it before writing any output, so the kernel can
    re-assemble the stage and factor it with dense Bunch-Kaufman pivoting instead."""
    be, _ = MODELS[name]()
    gen = be.problem.gen
    ni, nv, nx, nc = _dims(gen)
    rng = np.random.default_rng(3)
    A = _random_system(gen, rng)
    p, q = next(b for b in gen.elim.blocks if len(b) == 2)
    A[p, :] = 0.0
    A[:, p] = 0.0
    out = elim_sim.run(elim_sim.compile_body(gen.elim_lines), elim_sim.compact(A, gen.compact), ni, nx + nc + 2,
                       nx * nx + nc * nc + nc * nx, nx + nc)
    assert out["bad"]
    assert np.isnan(out["TR"]).all()


def test_static_plan_is_sparse():
    """The plan touches far fewer entries than the dense elimination (one_room: the
    structure has 14 interior pivots; dense BK updates 812 entries per stage)."""
    be, _ = MODELS["one_room"]()
    pl = be.problem.gen.elim
    assert len({i for b in pl.blocks for i in b}) == 14
    assert pl.n_update < 100


def test_mhe_stage0_plan_pivots_open_rows_alone():
    """MHE stage 0: the link rows of the free x_0 / parameters are open (bounds +-1e8), so
    their KKT diagonal is huge; the stage-0 plan takes them as 1x1 pivots (the generic
    plan pairs them with the copies xi_0, theta_0 and its 2x2 pivots fail the growth bound,
    which sent stage 0 to the dense path on every factorisation) and stays accurate with
    a 1e16 diagonal on those rows."""
    from agentlib_mpc_amd.runtime import codegen

    be, _ = MODELS["mhe_room"]()
    gen, nlp = be.problem.gen, be.problem.nlp
    eq, eq0 = codegen.equality_rows(nlp), codegen.equality_rows(nlp, stage=0)
    open_rows = sorted(gen.crow[r] for r in set(eq) - set(eq0))
    assert open_rows
    in_pairs = {i for b in gen.elim0.blocks if len(b) == 2 for i in b}
    assert not in_pairs & set(open_rows)
    assert {i for b in gen.elim.blocks if len(b) == 2 for i in b} & set(open_rows)
    ni, nv, nx, nc = _dims(gen)
    ntr = nx + nc + 1
    rng = np.random.default_rng(5)
    A = _random_system(gen, rng, gen.elim0)
    for r in open_rows:
        A[r, r] = -1e16
    out = elim_sim.run(elim_sim.compile_body(gen.elim0_lines), elim_sim.compact(A, gen.compact), ni, ntr,
                       nx * nx + nc * nc + nc * nx, nx + nc)
    assert not out["bad"]
    W = np.linalg.solve(A[:ni, :ni], A[:ni, ni:])
    np.testing.assert_allclose(out["TR"].reshape(ntr, ni).T, W, rtol=1e-8, atol=1e-8 * np.abs(W).max())
