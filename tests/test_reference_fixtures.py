"""The reference's own test expectations on its own test-suite fixtures (CPU).

`tests/fixtures/casadi_test_model.py` (loaded from /root/reference through the backend's
``{"file", "class_name"}`` model injection, as the reference's `tests/conftest.py:6-15`
does with agentlib's ``custom_injection``) and the assertions of
`tests/test_casadi_backend.py:61-161` and `tests/test_mpc.py:151-196`, restated against this
package's variable groups, systems, transcription and backend:

* ``OptimizationVariable.declare`` raises ValueError for an incomplete or foreign ref list;
* a ``BaseSystem`` holds 7 quantities, 3 parameter and 4 variable groups;
* the collocation state grid has (d+1)N+1 points starting at 0;
* ``add_opt_var`` of the controls at two prediction times gives the grid [0, 10];
* the backend's bound vectors match its variable and constraint counts;
* ``BadNamesModel`` raises NameError and ``InstanceAttributeSetterTestModel`` AttributeError
  when the backend builds them.

The solve of `test_mpc.py:151-162` (``len(result["myctrl"]) == 5``) needs the GPU and is in
tests/test_gpu_fixtures.py, with this package's restatement of the fixture model
(`models/examples.FixtureModel`), which the last test here checks against the file.
"""

import math
import pathlib

import numpy as np
import pytest

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.data_structures.mpc_datamodels import CasadiDiscretizationOptions, VariableReference
from agentlib_mpc_amd.models.casadi_model import CasadiState
from agentlib_mpc_amd.optimization_backends import create_optimization_backend
from agentlib_mpc_amd.optimization_backends.backend import custom_injection
from agentlib_mpc_amd.optimization_backends.discretization import BasicCollocation, _Transcriber
from agentlib_mpc_amd.optimization_backends.mi355x import MI355XBaseBackend
from agentlib_mpc_amd.optimization_backends.system import BaseSystem, OptimizationVariable

FIXTURE = pathlib.Path("/root/reference/tests/fixtures/casadi_test_model.py")


def test_optimization_variable():
    """`test_casadi_backend.py:61-93`."""
    variables = [CasadiState(name="s1", value=10, ub=10, lb=0), CasadiState(name="s2", lb=0)]
    with pytest.raises(ValueError):
        OptimizationVariable.declare(denotation="state", variables=variables, ref_list=["s1"],
                                     assert_complete=True)
    OptimizationVariable.declare(denotation="state", variables=variables, ref_list=["s1"])
    v2 = OptimizationVariable.declare(denotation="state", variables=variables, ref_list=["s1", "s2"],
                                      use_in_stage_function=False)
    assert v2.ref_names == v2.full_names
    with pytest.raises(ValueError):
        OptimizationVariable.declare(denotation="state", variables=variables, ref_list=["s3"])


needs_fixture = pytest.mark.skipif(not FIXTURE.is_file(), reason="reference fixtures not present")


@pytest.fixture
def model_type():
    return {"file": str(FIXTURE), "class_name": "MyCasadiModel"}


@pytest.fixture
def var_ref():
    """`test_casadi_backend.py:25-33`."""
    return VariableReference(states=["state"], controls=["myctrl"], inputs=["disturbance"],
                             parameters=["par", "par2"], outputs=["myout"])


@pytest.fixture
def example_casadi_system(model_type, var_ref):
    model = custom_injection(model_type)()
    sys_ = BaseSystem()
    sys_.initialize(model=model, var_ref=var_ref)
    return sys_


@needs_fixture
def test_system(example_casadi_system):
    """`test_casadi_backend.py:96-109`."""
    s = example_casadi_system
    assert len(s.quantities) == 7
    assert len(s.parameters) == 3
    assert len(s.variables) == 4
    assert "initial_" + s.states.name == s.initial_state.name
    assert s.initial_state.use_in_stage_function is False
    assert len(s.model_parameters.full_names) == len(s.model_parameters.full_symbolic)


@needs_fixture
def test_discretization(example_casadi_system):
    """`test_casadi_backend.py:112-132`: the collocation state grid."""
    s = example_casadi_system
    opts = CasadiDiscretizationOptions()
    nlp = BasicCollocation(options=opts).transcribe(s)
    assert all(g in nlp.var_groups for g in (s.states.name, s.controls.name, s.algebraics.name, s.outputs.name))
    grid = nlp.var_groups[s.states.name].grid
    assert grid[0] == 0
    assert len(grid) == (opts.collocation_order + 1) * opts.prediction_horizon + 1


@needs_fixture
def test_add_opt(example_casadi_system):
    """`test_casadi_backend.py:135-151`."""
    s = example_casadi_system
    t = _Transcriber(CasadiDiscretizationOptions())
    assert any([t.var_groups, t.par_groups, t.w]) is False
    t.add_opt_var(s.states)
    assert all([t.w, t.var_groups])
    assert any([t.p, t.par_groups]) is False
    t.add_opt_par(s.model_parameters)
    assert all([t.p, t.par_groups])
    t.add_opt_var(s.controls)
    t.pred_time += 10
    t.add_opt_var(s.controls)
    assert t.var_groups[s.controls.name].grid == [0, 10]


@needs_fixture
def test_create_backend(model_type, var_ref):
    """`test_casadi_backend.py:154-161`: bounds of the constraints and variables match their
    counts (backend ``casadi_basic`` with default options)."""
    be = MI355XBaseBackend(config={"model": {"type": model_type}})
    be.setup_optimization(var_ref)
    nlp = be.problem.nlp
    assert len(nlp.g_lb) == len(nlp.g_ub) == len(nlp.g_exprs)
    cv = {n: bm.V(n, v) for n, v in (("state", 298.16), ("myctrl", 0.02), ("disturbance", 270.0),
                                      ("par", 12.0), ("par2", 10.0), ("myout", None))}
    p, lbw, ubw, w0 = be.problem.marshal.inputs([cv], 0.0, None)
    assert lbw.shape[1] == ubw.shape[1] == nlp.nw
    assert p.shape[1] == nlp.npar
    assert nlp.ng_total == len(nlp.g_exprs)


def _mpc_backend(class_name):
    """The MPC module test's backend config (`test_mpc.py:121-146`) with another fixture class
    and the module's variable lists emptied, as `test_mpc.py:172-196` does."""
    be = create_optimization_backend({
        "type": "casadi",
        "model": {"type": {"file": str(FIXTURE), "class_name": class_name}},
        "discretization_options": {"prediction_horizon": 5, "time_step": 900},
    })
    be.setup_optimization(VariableReference(states=[], controls=[], inputs=[], parameters=[], outputs=[]))
    return be


@needs_fixture
def test_bad_names():
    """`test_mpc.py:172-184`: parameters named ``system`` and ``time`` are rejected."""
    with pytest.raises(NameError):
        _mpc_backend("BadNamesModel")


@needs_fixture
def test_instance_setter():
    """`test_mpc.py:186-196`: assigning a model variable as an instance attribute is rejected."""
    with pytest.raises(AttributeError, match="instance attribute with the name myout"):
        _mpc_backend("InstanceAttributeSetterTestModel")


@needs_fixture
def test_restated_fixture_model_gives_the_files_nlp():
    """The GPU fixture solve uses ``models/examples.FixtureModel``; it must be the file's model."""
    ours, _ = bm.fixture_mpc()
    theirs, _ = bm.fixture_mpc(model={"type": {"file": str(FIXTURE), "class_name": "MyCasadiModel"}})
    assert ours.problem.nlp.nlp_dims() == theirs.problem.nlp.nlp_dims() == {"nw": 41, "ng": 35, "np": 19}
    assert ours.problem.gen.source == theirs.problem.gen.source
    ours, _ = bm.fixture_admm()
    theirs, _ = bm.fixture_admm(model={"type": {"file": str(FIXTURE), "class_name": "MyCasadiModel"}})
    assert ours.problem.gen.source == theirs.problem.gen.source


def test_fixture_marshalling_matches_the_oracle_restatement():
    """The MPC-test config marshals to exactly the oracle's hand-written NLP inputs."""
    from tests import configs

    case = configs.fixture_mpc()
    p, lbw, ubw, w0 = case.backend.problem.marshal.inputs([case.current_vars], 0.0, None)
    op, olb, oub, ow0 = case.oracle_inputs
    np.testing.assert_array_equal(p[0], op)
    np.testing.assert_array_equal(lbw[0], olb)
    np.testing.assert_array_equal(ubw[0], oub)
    np.testing.assert_array_equal(w0[0], ow0)
    assert math.isclose(case.backend.problem.nlp.ts, 900.0)
