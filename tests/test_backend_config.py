"""Backend configuration (CPU): solver selection and option mapping.

Reference: ``SolverFactory`` (`data_structures/casadi_utils.py:120-217`): IPOPT
defaults max_iter=100, tol=1e-4, user options merged from ``options["ipopt"]``;
fatrop options from ``options["fatrop"]`` with the same defaults; an unknown
solver name raises ``ValueError``.
"""

import pytest

from agentlib_mpc_amd.optimization_backends import create_optimization_backend
from agentlib_mpc_amd.optimization_backends.mi355x import ipopt_options_to_kernel


def _backend(solver):
    return create_optimization_backend({
        "type": "casadi", "model": {"type": "agentlib_mpc_amd.models.examples.OneRoom"}, "solver": solver})


def test_reference_defaults_and_overrides():
    assert ipopt_options_to_kernel({}) == {"max_iter": 100, "tol": 1e-4}
    assert ipopt_options_to_kernel({"ipopt": {"tol": 1e-8}, "ipopt.max_iter": 7}) == {"max_iter": 7, "tol": 1e-8}
    # IPOPT options the kernel has no counterpart for are accepted and ignored
    assert ipopt_options_to_kernel({"ipopt": {"print_level": 0, "linear_solver": "ma27"}}) == {
        "max_iter": 100, "tol": 1e-4}


def test_fatrop_configs_run_on_the_kernel():
    be = _backend({"name": "fatrop", "options": {"fatrop": {"tol": 1e-6, "max_iter": 40},
                                                 "structure_detection": "auto"}})
    assert be.solver_options == {"max_iter": 40, "tol": 1e-6}


@pytest.mark.parametrize("name", ["osqp", "qpoases", "sqpmethod", "gurobi", "bonmin", "proxqp"])
def test_non_interior_point_solvers_are_rejected(name):
    with pytest.raises(ValueError, match="not available"):
        _backend({"name": name})
