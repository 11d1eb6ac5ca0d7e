"""Import aliases for model files written against the reference package.

User models are ordinary Python files that import the reference's model API,
``from agentlib_mpc.models.casadi_model import CasadiModel, CasadiState, ...``
(e.g. `examples/one_room_mpc/physical/simple_mpc.py:8-15`,
`examples/exchange_admm/models/room_model.py:1-8`), and are injected by the MPC module
through ``{"file": ..., "class_name": ...}`` (`modules/mpc/mpc.py:110-143`, agentlib
``custom_injection``).  When the real ``agentlib_mpc`` is not installed, the modules those
files import resolve to this package's restatements of the same API, so the files load
unchanged.  Nothing is aliased when the reference package itself is importable.
"""

from __future__ import annotations

import importlib
import importlib.util
import sys
import types

#: reference module -> this package's restatement of its model API
ALIASES = {
    "agentlib_mpc.models.casadi_model": "agentlib_mpc_amd.models.casadi_model",
    "agentlib_mpc.models.casadi_ml_model": "agentlib_mpc_amd.models.casadi_ml_model",
    "agentlib_mpc.models.casadi_predictor": "agentlib_mpc_amd.models.casadi_predictor",
    "agentlib_mpc.models.serialized_ml_model": "agentlib_mpc_amd.models.serialized_ml_model",
    "agentlib_mpc.data_structures.objective": "agentlib_mpc_amd.data_structures.objective",
    "agentlib_mpc.data_structures.ml_model_datatypes": "agentlib_mpc_amd.data_structures.ml_model_datatypes",
    "agentlib_mpc.data_structures.mpc_datamodels": "agentlib_mpc_amd.data_structures.mpc_datamodels",
}
_installed = False


def reference_available() -> bool:
    if _installed:
        return False
    try:
        return importlib.util.find_spec("agentlib_mpc") is not None
    except (ImportError, ValueError):
        return False


def install_reference_aliases() -> bool:
    """Alias the reference's model-API modules to this package (once; no-op when the
    reference is installed).  Returns True if the aliases are in place."""
    global _installed
    if _installed:
        return True
    if reference_available():
        return False
    for name, target in ALIASES.items():
        parts = name.split(".")
        for i in range(1, len(parts)):
            pkg = ".".join(parts[:i])
            if pkg not in sys.modules:
                mod = types.ModuleType(pkg)
                mod.__path__ = []  # namespace-like: only the aliased submodules exist
                sys.modules[pkg] = mod
        module = importlib.import_module(target)
        sys.modules[name] = module
        parent, _, leaf = name.rpartition(".")
        setattr(sys.modules[parent], leaf, module)
    _installed = True
    return True
