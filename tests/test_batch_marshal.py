"""Vectorised batch marshalling (CPU): :class:`BatchMarshal` against the per-agent
restatement of the reference input path (`CompiledProblem.mpc_inputs` /
`initial_guess` / `nlp_inputs`, `core/casadi_backend.py:141-253`,
`core/discretization.py:212-348`) and of the result matrix (:360-484), bit for bit."""

import copy

import numpy as np
import pandas as pd
import pytest

from tests import configs


def _agents(case, n, seed):
    """n distinct agents: scalar values perturbed, one trajectory given as a list and one
    as a time series (sampled per agent)."""
    rng = np.random.default_rng(seed)
    out = []
    prob = case.backend.problem
    for a in range(n):
        cv = copy.deepcopy(case.current_vars)
        for name, v in cv.items():
            if isinstance(v.value, (float, int)) and not isinstance(v.value, bool):
                v.value = float(v.value) * (1.0 + 0.01 * rng.standard_normal())
        out.append(cv)
    # one parameter trajectory as a list / series on some agents
    for par in prob.system.parameters:
        lay = prob.nlp.par_groups.get(par.name)
        refs = [n for n in par.full_names if n in par.ref_names]
        if lay is None or not refs or len(lay.grid) < 3:
            continue
        name, grid = refs[0], list(lay.grid)
        out[0][name].value = [float(x) for x in rng.uniform(1, 2, len(grid))]
        if n > 1:
            out[1][name].value = pd.Series(rng.uniform(1, 2, 4), index=[-100.0, 0.0, 500.0, 2e4])
        break
    return out


@pytest.mark.parametrize("name", ["one_room", "admm_room", "exchange_supply", "room_nn", "mhe_room",
                                  "one_room_du", "tz_cca"])
def test_batch_marshal_matches_per_agent_path(name):
    case = configs.CASES[name]()
    prob = case.backend.problem
    agents = _agents(case, 5, 1)
    rng = np.random.default_rng(2)
    w_prev = rng.uniform(0.0, 1.0, (5, prob.nlp.nw))
    w_prev[3] = np.nan  # no previous optimum for agent 3
    p, lbw, ubw, w0, (slb, sub) = prob.marshal.inputs(agents, 30.0, w_prev, return_sampled_bounds=True)
    for a, cv in enumerate(agents):
        mi = prob.mpc_inputs(cv, 30.0)
        rem = None if a == 3 else prob.outputs(w_prev[a])
        mi.update(prob.initial_guess(mi, rem))
        want = prob.nlp_inputs(mi)
        for got, ref in zip((p[a], lbw[a], ubw[a], w0[a]), want):
            np.testing.assert_array_equal(got, ref)
        w = w_prev[a:a + 1] if a != 3 else w0[a:a + 1]
        mat = prob.marshal.result_matrices(p[a:a + 1], slb[a:a + 1], sub[a:a + 1], w)[0]
        ref_mat = prob.result_matrix(mi, w_prev[a] if a != 3 else w0[a])
        np.testing.assert_array_equal(np.isnan(mat), np.isnan(ref_mat))
        np.testing.assert_array_equal(np.nan_to_num(mat), np.nan_to_num(ref_mat))


def test_batch_marshal_errors_like_the_reference():
    case = configs.one_room()
    prob = case.backend.problem
    cv = copy.deepcopy(case.current_vars)
    name = next(n for p_ in prob.system.parameters for n in p_.full_names if n in p_.ref_names)
    cv[name].value = None
    with pytest.raises(ValueError, match="empty"):
        prob.marshal.inputs([case.current_vars, cv], 0.0)
    cv[name].value = [1.0, 2.0]  # wrong length (`utils/sampling.py:84-91`)
    with pytest.raises(ValueError):
        prob.marshal.inputs([cv], 0.0)
