"""Resident plugin batch (CPU): the incremental device-resident inputs of
``MI355XBackend.solve_batch`` (`optimization_backends/plugin_batch.py`) equal a full
re-marshalling of the agents' variables (`problem.BatchMarshal.inputs`, the reference's
input path `core/casadi_backend.py:141-253`, `core/discretization.py:212-348`) after
every kind of change: scalar measurements, a trajectory given as a list, bounds, and the
warm start with the parameter-derived guess; the per-agent result rows equal the
re-marshalled ones; empty values and non-MPCVariable inputs raise the reference's errors.
The device is the CPU here (torch tensors), the kernel is not called."""

import copy

import numpy as np
import pytest
import torch

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.optimization_backends.plugin_batch import ResidentBatch, RowSource


def _agents(cv, n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        c = copy.deepcopy(cv)
        c["T"].value = float(rng.uniform(291, 301))
        c["load"].value = float(rng.uniform(50, 250))
        c["mDot"].value = float(rng.uniform(0, 0.05))
        out.append(c)
    return out


def _check(rb, m, agents, now, w_prev):
    p, lbw, ubw, w0, (ls, us) = m.inputs(agents, now, w_prev, return_sampled_bounds=True)
    np.testing.assert_array_equal(rb.P.numpy(), p)
    np.testing.assert_array_equal(rb.L.numpy(), lbw)
    np.testing.assert_array_equal(rb.U.numpy(), ubw)
    np.testing.assert_array_equal(rb.W.numpy(), w0)
    return p, ls, us


@pytest.mark.parametrize("small", [True, False])
def test_resident_inputs_equal_full_marshalling(small, monkeypatch):
    """Both update paths: host mirrors + one upload (small batches) and device scatters."""
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    m = be.problem.marshal
    agents = _agents(cv, 16, 3)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    _check(rb, m, agents, 0.0, None)
    snaps = [RowSource(rb, rb.last)]
    want_rows = [m.inputs(agents, 0.0, None, return_sampled_bounds=True)]
    # step 2: new measurements, one agent's T_upper as a trajectory on its grid, a bound
    w_prev = rb.W.numpy().copy()
    w_prev[:, 5:9] += 0.25          # stands in for the solution the kernel would write in place
    rb.W.copy_(torch.from_numpy(w_prev))
    if rb.small:
        rb.hW[:] = w_prev  # what solve() does with the solution it reads back
    for i, c in enumerate(agents):
        c["T"].value += 0.1 * (i + 1)
    grid = len(be.problem.nlp.par_groups["d"].grid)
    agents[3]["T_upper"] = copy.deepcopy(agents[3]["T_upper"])
    agents[3]["T_upper"].value = list(np.linspace(294.0, 296.0, grid))
    agents[5]["mDot"] = copy.deepcopy(agents[5]["mDot"])
    agents[5]["mDot"].ub = 0.04
    snap = rb.update(agents, 300.0)
    _check(rb, m, agents, 300.0, w_prev)
    snaps.append(RowSource(rb, snap))
    want_rows.append(m.inputs(agents, 300.0, w_prev, return_sampled_bounds=True))
    # step 3: nothing changed -> nothing uploaded, same arrays
    before = {k: v for k, v in rb.last.items()}
    rb.update(agents, 300.0)
    assert all(rb.last[k] is before[k] for k in before)
    # the snapshots of both calls still give their own rows (later calls never modify them)
    for src, (p, _, _, _, (ls, us)) in zip(snaps, want_rows):
        for i in (0, 3, 5, 15):
            rp, rls, rus = src.rows(i)
            np.testing.assert_array_equal(rp, p[i])
            np.testing.assert_array_equal(rls, ls[i])
            np.testing.assert_array_equal(rus, us[i])


def test_resident_inputs_raise_the_reference_errors():
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    agents = _agents(cv, 4, 5)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    bad = [dict(a) for a in agents]
    bad[2]["load"] = copy.deepcopy(bad[2]["load"])
    bad[2]["load"].value = None
    with pytest.raises(ValueError, match="empty"):
        rb.update(bad, 0.0)

    class Plain:
        value, lb, ub = 150.0, -np.inf, np.inf

    bad = [dict(a) for a in agents]
    bad[1]["load"] = Plain()
    with pytest.raises(TypeError, match="interpolationmethod"):
        rb.update(bad, 0.0)


def test_native_reader_equals_python_reader():
    """The one-pass native attribute reader (``csrc/mpcx_pyread.c``) gives the Python
    reader's columns for every value kind the agents may hold: floats, ints, numpy
    scalars, NaN, a trajectory list (those three take the Python path per column), and a
    missing variable raises KeyError."""
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    agents = _agents(cv, 9, 8)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    grid = len(be.problem.nlp.par_groups["d"].grid)
    for i, c in enumerate(agents):
        for k in c:
            c[k] = copy.deepcopy(c[k])
    agents[1]["load"].value = 120            # int
    agents[2]["T_in"].value = np.float64(290.5)  # numpy scalar
    agents[3]["mDot"].lb = 0                  # int bound
    agents[4]["T_upper"].value = list(np.linspace(294.0, 296.0, grid))
    agents[6]["mDot"].ub = np.nan             # NaN bound
    got = rb.read(agents, 300.0)
    want = rb._read_python(agents, 300.0, rb.refs)
    assert got.keys() == want.keys()
    for key in want:
        g, w = got[key], want[key]
        if isinstance(w, dict):
            assert isinstance(g, dict) and g.keys() == w.keys()
            for gid in w:
                np.testing.assert_array_equal(g[gid], w[gid])
        else:
            np.testing.assert_array_equal(g, w)
    del agents[5]["load"]
    with pytest.raises(KeyError):
        rb.read(agents, 300.0)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
def test_gpu_resident_plugin_path_matches_host_marshalling(small, monkeypatch):
    """Three closed-loop steps through ``solve_batch`` (resident inputs, warm start in HBM)
    against the host path (full re-marshalling with the previous optimum as guess,
    ``solve_arrays``): identical solutions, statuses and per-agent Results -- with the
    small-batch update (host mirrors, one upload) and with the device scatters."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    twin = bm.one_room(solver_options=bm.REFERENCE)[0]
    agents = _agents(cv, 24, 11)
    m = twin.problem.marshal
    w_prev = None
    rng = np.random.default_rng(2)
    for step in range(3):
        if step:
            for c in agents:
                c["T"].value += float(rng.normal(0.0, 0.3))
            agents[7]["load"] = copy.deepcopy(agents[7]["load"])
            agents[7]["load"].value = list(np.linspace(80.0, 220.0, len(twin.problem.nlp.par_groups["d"].grid)))
        res = be.solve_batch(300.0 * step, agents)
        p, lbw, ubw, w0, sampled = m.inputs(agents, 300.0 * step, w_prev, return_sampled_bounds=True)
        ref = twin.solve_arrays(p, lbw, ubw, w0, result_bounds=sampled)
        w_prev = ref.w.copy()
        np.testing.assert_array_equal(res.stats.array["status"], ref.stats.array["status"])
        np.testing.assert_array_equal(res.stats.array["iter_count"], ref.stats.array["iter_count"])
        np.testing.assert_allclose(res.w, ref.w, rtol=1e-13, atol=1e-13)
        for i in (0, 7, 23):
            np.testing.assert_allclose(res[i].matrix, ref[i].matrix, rtol=1e-13, atol=1e-13, equal_nan=True)


@pytest.mark.parametrize("small", [True, False])
def test_cold_restart_guess_equals_full_marshalling(small, monkeypatch):
    """``restart_cold`` (a backend's first solve, `core/discretization.py:212-245`): the next
    update's guess equals the full marshalling's cold guess -- small batches build it from
    the host mirrors, large ones re-marshal the rows."""
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    m = be.problem.marshal
    agents = _agents(cv, 6, 4)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    rb.W.fill_(1.5)
    if rb.small:
        rb.hW[:] = 1.5
    for i, c in enumerate(agents):
        c["T"].value += 0.3 * i
    agents[2]["mDot"] = copy.deepcopy(agents[2]["mDot"])
    agents[2]["mDot"].ub = 0.03
    rb.restart_cold()
    rb.update(agents, 600.0)
    _check(rb, m, agents, 600.0, None)


def test_native_reader_takes_any_mapping():
    """Agents' variable sets given as mappings that are not dicts (the native reader's
    ``PyObject_GetItem`` path) read the same as dicts."""
    from collections.abc import Mapping

    class Vars(Mapping):
        def __init__(self, d):
            self.d = d

        def __getitem__(self, k):
            return self.d[k]

        def __iter__(self):
            return iter(self.d)

        def __len__(self):
            return len(self.d)

    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    agents = _agents(cv, 5, 9)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    want = rb.read(agents, 0.0)
    got = rb.read([Vars(a) for a in agents], 0.0)
    assert got.keys() == want.keys()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k])


@pytest.mark.parametrize("small", [True, False])
def test_nan_input_after_the_first_call_raises_like_the_host_path(small, monkeypatch):
    """A NaN measurement or bound arriving at a later call is rejected before any launch with
    the host path's error (`BatchMarshal.assemble`: 'incomplete NLP inputs'), and the next
    valid call re-applies every column."""
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    m = be.problem.marshal
    agents = _agents(cv, 6, 11)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    for field, attr in (("T", "value"), ("mDot", "ub")):
        bad = [copy.deepcopy(a) for a in agents]
        setattr(bad[2][field], attr, float("nan"))
        with pytest.raises(ValueError, match="incomplete NLP inputs"):
            m.inputs(bad, 300.0, None)                 # the host path
        with pytest.raises(ValueError, match="incomplete NLP inputs"):
            rb.update(bad, 300.0)                      # the resident plugin path
    # the agents' valid values again: every column re-applied, no NaN left behind
    rb.update(agents, 300.0)
    w_prev = rb.W.numpy().copy()
    _check(rb, m, agents, 300.0, w_prev)


@pytest.mark.parametrize("small", [True, False])
def test_warm_starts_follow_the_agent_keys(small, monkeypatch):
    """``solve_batch(..., agent_ids)`` plumbing: after a permutation of
    the batch every agent keeps ITS previous optimum (the reference's one remembered solution
    per backend, `core/discretization.py:221-223`), a new key starts cold, and the inputs
    equal a full re-marshalling of the permuted agents with those warm starts."""
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    m = be.problem.marshal
    agents = _agents(cv, 5, 21)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    sol = rb.W.numpy().copy() + np.arange(5)[:, None] * 0.01 + 0.3   # stands in for the solutions
    rb.W.copy_(torch.from_numpy(sol))
    if rb.small:
        rb.hW[:] = sol
    src = np.array([2, 0, -1, 1, 4])          # entry 2 is a new agent
    newcomer = copy.deepcopy(cv)
    newcomer["T"].value = 299.5
    perm = [agents[2], agents[0], newcomer, agents[1], agents[4]]
    rb.permute_warm_starts(src)
    rb.update(perm, 300.0)
    w_prev = np.full_like(sol, np.nan)
    w_prev[src >= 0] = sol[src[src >= 0]]
    _check(rb, m, perm, 300.0, w_prev)
    # a new batch size: known agents carry their optima over, the others start cold
    rb2 = ResidentBatch(be.problem, None, perm[:3], 300.0, torch.device("cpu"))
    rb2.adopt_warm_starts(rb, np.array([4, -1, 0]))
    want = m.inputs(perm[:3], 300.0, None)[3]
    want[0], want[2] = rb.W.numpy()[4], rb.W.numpy()[0]
    np.testing.assert_array_equal(rb2.W.numpy(), want)


@pytest.mark.parametrize("small", [True, False])
def test_failed_agent_restarts_cold_after_permutation(small, monkeypatch):
    """an agent whose last solve came back NaN (``cold_rows``, old slot numbering)
    restarts cold wherever the next call puts it -- after a permutation of the batch and after
    a change of batch size -- and the agent now sitting in its old slot keeps its own warm start."""
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    m = be.problem.marshal
    agents = _agents(cv, 5, 23)
    rb = ResidentBatch(be.problem, None, agents, 0.0, torch.device("cpu"))
    sol = rb.W.numpy().copy() + np.arange(5)[:, None] * 0.01 + 0.3
    sol[1] = np.nan                            # agent 1's solve failed (what solve() records)
    rb.W.copy_(torch.from_numpy(sol))
    if rb.small:
        rb.hW[:] = sol
    rb.cold_rows = np.array([1])
    src = np.array([1, 3, 4, 0, 2])            # agent 1 moves to slot 0; agent 3 into its old slot
    perm = [agents[i] for i in src]
    rb.permute_warm_starts(src)
    rb.update(perm, 300.0)
    w_prev = sol[src].copy()                   # NaN row = cold start in the host marshalling
    _check(rb, m, perm, 300.0, w_prev)
    assert np.isfinite(rb.W.numpy()).all()
    # a failure, then a batch-size change: the failed agent keeps the cold guess
    sol2 = rb.W.numpy().copy() + 0.1
    sol2[2] = np.nan
    rb.W.copy_(torch.from_numpy(sol2))
    if rb.small:
        rb.hW[:] = sol2
    rb.cold_rows = np.array([2])
    rb2 = ResidentBatch(be.problem, None, [perm[2], perm[4]], 600.0, torch.device("cpu"))
    rb2.adopt_warm_starts(rb, np.array([2, 4]))
    want = m.inputs([perm[2], perm[4]], 600.0, None)[3]
    want[1] = sol2[4]
    np.testing.assert_array_equal(rb2.W.numpy(), want)


@pytest.mark.gpu
@pytest.mark.parametrize("small", [True, False])
def test_gpu_permuted_batch_keeps_each_agents_warm_start(small, monkeypatch):
    """a batch permuted between two calls (``agent_ids``) equals two
    unpermuted calls agent by agent -- same statuses, iteration counts and solutions -- and
    a batch of another size carries the known agents' optima over."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from agentlib_mpc_amd.optimization_backends import plugin_batch

    monkeypatch.setattr(plugin_batch, "SMALL_BATCH", 64 if small else 0)
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    twin = bm.one_room(solver_options=bm.REFERENCE)[0]
    agents = _agents(cv, 12, 5)
    ids = [f"room{i}" for i in range(12)]
    be.solve_batch(0.0, agents, agent_ids=ids)
    twin.solve_batch(0.0, agents, agent_ids=ids)
    for c in agents:
        c["T"].value += 0.2
    perm = np.random.default_rng(4).permutation(12)
    got = be.solve_batch(300.0, [agents[i] for i in perm], agent_ids=[ids[i] for i in perm])
    want = twin.solve_batch(300.0, agents, agent_ids=ids)
    np.testing.assert_array_equal(got.stats.array["iter_count"], want.stats.array["iter_count"][perm])
    np.testing.assert_array_equal(got.stats.array["status"], want.stats.array["status"][perm])
    np.testing.assert_allclose(got.w, want.w[perm], rtol=1e-13, atol=1e-13)
    # a smaller batch of known agents in another order: the same warm starts again
    sub = perm[:5]
    for c in agents:
        c["T"].value += 0.2
    got = be.solve_batch(600.0, [agents[i] for i in sub], agent_ids=[ids[i] for i in sub])
    want = twin.solve_batch(600.0, agents, agent_ids=ids)
    np.testing.assert_array_equal(got.stats.array["iter_count"], want.stats.array["iter_count"][sub])
    np.testing.assert_allclose(got.w, want.w[sub], rtol=1e-13, atol=1e-13)
