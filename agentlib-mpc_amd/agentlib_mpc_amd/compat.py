"""Loading model files written against the reference package.

User models are ordinary Python files that import the reference's model API,
``from agentlib_mpc.models.casadi_model import CasadiModel, CasadiState, ...``
(e.g. `examples/one_room_mpc/physical/simple_mpc.py:8-15`,
`examples/exchange_admm/models/room_model.py:1-8`), and are injected by the MPC module
through ``{"file": ..., "class_name": ...}`` (`modules/mpc/mpc.py:110-143`, agentlib
``custom_injection``) or named as a class / dotted path.  The backend needs the model
traced by :mod:`agentlib_mpc_amd.symbolic`, so these imports must resolve to this
package's restatement of the same API.  Two modes:

* **reference not installed** -- :func:`install_reference_aliases` puts the aliased module
  names into ``sys.modules`` (nothing else could claim them), so model files load
  unchanged wherever they are imported from.
* **reference installed** (the deployment mode: agentlib, casadi and ``agentlib_mpc``
  are importable) -- nothing global is touched.  The model's file is executed a second
  time, privately, by :func:`load_model_file`: its module namespace gets a
  ``__builtins__`` whose ``__import__`` resolves the aliased names (and ``casadi``) to
  this package and passes every other import through.  A model class that was already
  imported normally (a class object or dotted path in the config, or an injected file the
  reference loaded) is re-read from its source file the same way
  (:func:`retrace_model_class`); the user's reference-side class is never instantiated.
"""

from __future__ import annotations

import builtins
import importlib
import importlib.util
import inspect
import pathlib
import sys
import types
from typing import Dict, Optional

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
#: reference modules whose classes are model classes (a class deriving from one of
#: these is a reference-side model and must be re-read through the private map)
MODEL_BASES = {("agentlib_mpc.models.casadi_model", "CasadiModel"),
               ("agentlib_mpc.models.casadi_ml_model", "CasadiMLModel")}
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


# ---------------------------------------------------------------------------
# private import map (reference installed)
# ---------------------------------------------------------------------------
def _casadi_module() -> types.ModuleType:
    """``import casadi as ca`` inside a model file: the tracer's stand-in functions."""
    from agentlib_mpc_amd.models.casadi_model import ca

    mod = types.ModuleType("casadi")
    for k in dir(ca):
        if not k.startswith("_"):
            setattr(mod, k, getattr(ca, k))
    return mod


class _Package(types.ModuleType):
    """A package node of the private map: aliased children are attributes, anything
    else is read from the real (reference) package of the same name."""

    def __getattr__(self, item):
        real = importlib.import_module(self.__name__)
        return getattr(real, item)


class PrivateImportMap:
    """``__import__`` for one model file: aliased names -> this package, the rest as usual."""

    def __init__(self):
        self.targets: Dict[str, types.ModuleType] = {
            name: importlib.import_module(target) for name, target in ALIASES.items()}
        self.targets["casadi"] = _casadi_module()
        self.packages: Dict[str, _Package] = {}
        for name, module in self.targets.items():
            parts = name.split(".")
            for i in range(1, len(parts)):
                pkg = ".".join(parts[:i])
                self.packages.setdefault(pkg, _Package(pkg))
            if len(parts) > 1:
                parent = self.packages[".".join(parts[:-1])]
                object.__setattr__(parent, parts[-1], module)
        for pkg, node in self.packages.items():
            if "." in pkg:
                parent, _, leaf = pkg.rpartition(".")
                object.__setattr__(self.packages[parent], leaf, node)
        self._real = builtins.__import__

    def __call__(self, name, globals=None, locals=None, fromlist=(), level=0):
        if level == 0 and (name in self.targets or name in self.packages):
            if fromlist:
                return self.targets.get(name) or self.packages[name]
            top = name.partition(".")[0]
            return self.targets.get(top) or self.packages[top]
        return self._real(name, globals, locals, fromlist, level)

    def builtins(self) -> dict:
        b = dict(vars(builtins))
        b["__import__"] = self
        return b


def load_model_file(file, module_name: Optional[str] = None) -> types.ModuleType:
    """Execute a model file with the private import map (its ``agentlib_mpc`` model-API
    imports resolve to this package; nothing is registered in ``sys.modules`` under the
    reference's names)."""
    file = pathlib.Path(file).resolve()
    name = module_name or f"_mpcx_injected_{abs(hash(str(file)))}"
    if name in sys.modules:
        return sys.modules[name]
    source = file.read_text()
    module = types.ModuleType(name)
    module.__file__ = str(file)
    module.__builtins__ = PrivateImportMap().builtins()
    sys.modules[name] = module  # dataclasses / pydantic resolve annotations through it
    try:
        exec(compile(source, str(file), "exec"), module.__dict__)
    except BaseException:
        sys.modules.pop(name, None)
        raise
    return module


def is_reference_model_class(cls) -> bool:
    """True for a class deriving from the reference's (not this package's) model base."""
    if not isinstance(cls, type):
        return False
    return any((getattr(b, "__module__", None), b.__name__) in MODEL_BASES for b in inspect.getmro(cls))


def retrace_model_class(cls):
    """The same model class, read again from its source file through the private import
    map, so that it derives from this package's ``CasadiModel`` and can be traced."""
    file = inspect.getsourcefile(cls)
    if file is None:
        raise TypeError(f"model class {cls!r} has no source file to re-read for tracing")
    module = load_model_file(file)
    obj = module
    for part in cls.__qualname__.split("."):
        obj = getattr(obj, part)
    return obj
