"""Device-resident fleet session (optimization_backends/fleet_session.py).

CPU: the probed column maps reproduce the marshalling exactly -- updating a scalar
input in place gives the same kernel inputs as re-marshalling every agent's
``MPCVariable`` dict.  GPU: a closed loop through the session equals the plugin API
(``solve_batch``, warm start = each agent's previous optimum) step for step.
"""

import copy

import numpy as np
import pytest
import torch

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.optimization_backends.fleet_session import FleetSession


def _fleet(n, seed=5):
    be, cv = bm.one_room(solver_options=bm.REFERENCE)
    rng = np.random.default_rng(seed)
    agents = []
    for _ in range(n):
        c = copy.deepcopy(cv)
        c["T"].value = float(rng.uniform(292.0, 301.0))
        c["load"].value = float(rng.uniform(50.0, 250.0))
        agents.append(c)
    return be, cv, agents


def test_scalar_updates_match_remarshalling():
    be, cv, agents = _fleet(6)
    s = FleetSession(be, agents, device="cpu")
    rng = np.random.default_rng(1)
    newT, newload = rng.uniform(290.0, 303.0, 6), rng.uniform(20.0, 300.0, 6)
    s.update("T", newT)
    s.update("load", newload)
    for a, c in enumerate(agents):
        c["T"].value = float(newT[a])
        c["load"].value = float(newload[a])
    kp, kl, ku, _ = be.problem.to_kernel(*be.problem.marshal.inputs(agents, 0.0))
    np.testing.assert_array_equal(s.p.numpy(), kp)
    np.testing.assert_array_equal(s.lbw.numpy(), kl)
    np.testing.assert_array_equal(s.ubw.numpy(), ku)
    # initial state: parameter + x_0 bounds (kernel layout and the reference-layout copy)
    assert {k for k, _ in s.columns_of("T")} == {"p", "lbw", "ubw", "lbw_ref"}


def test_lifted_updates_keep_the_reference_layout_bounds():
    """NARX (lifted): inputs that fix past values the kernel NLP drops must reach the
    reference-layout bounds too, from which solution() rebuilds those variables."""
    be, cv = bm.room_nn(solver_options=bm.REFERENCE)
    agents = [copy.deepcopy(cv) for _ in range(3)]
    s = FleetSession(be, agents, device="cpu")
    names = ["T_air", "T_CCA_0"] + [k for k in cv if k.startswith("admm_lag_")]
    rng = np.random.default_rng(2)
    for name in names:
        new = rng.uniform(290.0, 300.0, 3)
        s.update(name, new)
        for a, c in enumerate(agents):
            c[name].value = float(new[a])
    _, lbw_ref, _, _ = be.problem.marshal.inputs(agents, 0.0)
    np.testing.assert_array_equal(s.lbw_ref, lbw_ref)


def test_update_rejects_wrong_shape_and_non_scalar_inputs():
    be, cv, agents = _fleet(3)
    s = FleetSession(be, agents, device="cpu")
    with pytest.raises(ValueError):
        s.update("T", np.zeros(4))
    agents[0]["load"].value = [100.0] * 5
    s2 = FleetSession.__new__(FleetSession)
    s2.__dict__.update(s.__dict__)
    s2._maps = {}
    s2.template = agents[0]
    with pytest.raises(TypeError):
        s2.columns_of("load")


@pytest.mark.gpu
def test_gpu_session_closed_loop_matches_plugin_api():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    be, cv, agents = _fleet(16)
    be2 = bm.one_room(solver_options=bm.REFERENCE)[0]  # plugin-API twin (own remembered guesses)
    sess = FleetSession(be, agents)
    rng = np.random.default_rng(3)
    for step in range(3):
        if step:
            meas = np.array([c["T"].value for c in agents]) + rng.normal(0.0, 0.2, len(agents))
            for a, c in enumerate(agents):
                c["T"].value = float(meas[a])
            sess.update("T", meas)
        sess.solve()
        res = be2.solve_batch(0.0, agents)
        np.testing.assert_allclose(sess.first_values("mDot"), res.first_values("mDot"), rtol=1e-12, atol=1e-14)
        st = sess.stats().array
        np.testing.assert_array_equal(st["iter_count"], res.stats.array["iter_count"])
        np.testing.assert_allclose(st["obj"], res.stats.array["obj"], rtol=1e-12)
        np.testing.assert_allclose(sess.solution(), res.w, rtol=1e-12, atol=1e-12)
