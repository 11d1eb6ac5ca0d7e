"""Backend registry (mirrors `agentlib_mpc/optimization_backends/__init__.py:6-72`).

The reference maps type strings to lazily imported classes.  The MI355X
backends register under their own keys and under the reference keys they
replace, so an agent config can switch by changing ``"type"`` only (or keep
it and point ``backend_types`` here).  A reference install can also load them
through its custom-injection path:
``{"type": {"file": ".../optimization_backends/mi355x.py", "class_name": "MI355XBackend"}}``.
"""

import importlib

from pydantic import BaseModel


class BackendImport(BaseModel):
    import_path: str
    class_name: str

    def __call__(self, *args, **kwargs):
        module = importlib.import_module(self.import_path)
        return getattr(module, self.class_name)(*args, **kwargs)


_MOD = "agentlib_mpc_amd.optimization_backends.mi355x"
_MHE = "agentlib_mpc_amd.optimization_backends.mhe"

backend_types = {
    "mi355x": BackendImport(import_path=_MOD, class_name="MI355XBackend"),
    "mi355x_basic": BackendImport(import_path=_MOD, class_name="MI355XBaseBackend"),
    "mi355x_admm": BackendImport(import_path=_MOD, class_name="MI355XADMMBackend"),
    "mi355x_ml": BackendImport(import_path=_MOD, class_name="MI355XMLBackend"),
    "mi355x_admm_ml": BackendImport(import_path=_MOD, class_name="MI355XADMMNNBackend"),
    "mi355x_mhe": BackendImport(import_path=_MHE, class_name="MHEBackend"),
    # drop-in aliases of the reference keys this backend replaces
    "casadi": BackendImport(import_path=_MOD, class_name="MI355XBackend"),
    "casadi_basic": BackendImport(import_path=_MOD, class_name="MI355XBaseBackend"),
    "casadi_admm": BackendImport(import_path=_MOD, class_name="MI355XADMMBackend"),
    "casadi_ml": BackendImport(import_path=_MOD, class_name="MI355XMLBackend"),
    "casadi_nn": BackendImport(import_path=_MOD, class_name="MI355XMLBackend"),
    "casadi_admm_ml": BackendImport(import_path=_MOD, class_name="MI355XADMMNNBackend"),
    "casadi_admm_nn": BackendImport(import_path=_MOD, class_name="MI355XADMMNNBackend"),
    "casadi_mhe": BackendImport(import_path=_MHE, class_name="MHEBackend"),
}

uninstalled_backend_types = {}


def create_optimization_backend(optimization_backend: dict, agent_id: str = None):
    """`modules/mpc/mpc.py:110-143` equivalent: resolve ``type`` and build the backend."""
    from agentlib_mpc_amd.optimization_backends.backend import OptimizationBackend, custom_injection

    cfg = dict(optimization_backend)
    _type = cfg.pop("type")
    cfg["name"] = agent_id
    if isinstance(_type, dict):
        backend = custom_injection(_type)(config=cfg)
    else:
        if _type not in backend_types:
            raise ValueError(f"Given backend type {_type!r} is not registered; registered: {sorted(backend_types)}")
        backend = backend_types[_type](config=cfg)
    assert isinstance(backend, OptimizationBackend)
    return backend
