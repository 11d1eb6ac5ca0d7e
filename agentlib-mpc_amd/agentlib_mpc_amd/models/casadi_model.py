"""User-facing symbolic model API, traced into :mod:`agentlib_mpc_amd.symbolic`.

Mirrors the reference's ``CasadiModel`` API (`agentlib_mpc/models/casadi_model.py`):
variable classes ``CasadiVariable``/``CasadiState``/``CasadiInput``/
``CasadiOutput``/``CasadiParameter`` (:36-296) with arithmetic overloads,
``CasadiModelConfig`` (:299-316) and ``CasadiModel`` (:323-584) with
``setup_system()``, ``.ode``/``.alg`` assignment, ``constraints`` as
``(lb, function, ub)`` tuples, ``get_constraints`` (:458-467),
``output_equations`` (:489-493), ``differentials``/``auxiliaries``
(:495-505) and the objective helpers (:516-545).

A model file written for the reference runs unchanged apart from the import
line (``from agentlib_mpc_amd.models.casadi_model import *``).  Simulation
(``do_step`` / integrators) belongs to the agentlib runtime and is not part of
this backend.
"""

from __future__ import annotations

import copy
import math
import warnings
from typing import Any, Dict, List, Optional, Tuple, Union  # noqa: F401 (re-exported for model files)

import numpy as np
import pydantic
from pydantic import ConfigDict, Field

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.symbolic import (  # noqa: F401  (model files use these names)
    exp, log, sqrt, tanh, sin, cos, fabs, fmax, fmin, if_else,
)

__all__ = [
    "CasadiVariable", "CasadiState", "CasadiInput", "CasadiOutput", "CasadiParameter",
    "CasadiModelConfig", "CasadiModel", "ModelConstraint", "List", "Optional", "Union",
    "exp", "log", "sqrt", "tanh", "sin", "cos", "fabs", "fmax", "fmin", "if_else", "ca",
]


class _CaNamespace:
    """Tiny stand-in for the ``casadi`` functions model files call (``ca.exp`` …)."""

    exp = staticmethod(sx.exp)
    log = staticmethod(sx.log)
    sqrt = staticmethod(sx.sqrt)
    tanh = staticmethod(sx.tanh)
    sin = staticmethod(sx.sin)
    cos = staticmethod(sx.cos)
    fabs = staticmethod(sx.fabs)
    fmax = staticmethod(sx.fmax)
    fmin = staticmethod(sx.fmin)
    if_else = staticmethod(sx.if_else)
    inf = math.inf

    @staticmethod
    def sum1(x):
        return sx.sum1(x)

    @staticmethod
    def vertcat(*xs):
        return [sx.as_expr(x) for x in xs]


ca = _CaNamespace()


class ModelConstraint(Tuple):
    pass


def _sym_of(x):
    return x.sym if isinstance(x, CasadiVariable) else x


class CasadiVariable:
    """Model variable with a scalar symbol (`casadi_model.py:36-152`)."""

    _causality = "local"

    def __init__(self, *, name: str, value: Any = None, unit: str = None,
                 description: str = None, lb: float = -math.inf, ub: float = math.inf,
                 type: str = None, alias: str = None, source: Any = None,
                 interpolation_method: str = "linear", **extra):
        self.name = name
        self.value = value
        self.unit = unit
        self.description = description
        self.lb = -math.inf if lb is None else lb
        self.ub = math.inf if ub is None else ub
        self.type = type
        self.alias = alias if alias is not None else name
        self.source = source
        self.interpolation_method = interpolation_method
        self.extra = extra
        shape = np.shape(value) if value is not None and not isinstance(value, (int, float)) else ()
        if shape not in ((), (1,), (1, 1)):
            raise NotImplementedError(
                f"Variable '{name}' has non-scalar value of shape {shape}; only scalar "
                "model variables are supported by this backend."
            )
        self._sym = sx.sym(name)

    def fresh_copy(self) -> "CasadiVariable":
        other = copy.copy(self)
        other.extra = dict(self.extra)
        other._sym = sx.sym(self.name)
        return other

    def update(self, **fields):
        for k, v in fields.items():
            if k == "name":
                continue
            if k in ("lb", "ub") and v is None:
                v = -math.inf if k == "lb" else math.inf
            setattr(self, k, v)

    @property
    def sym(self) -> sx.Expr:
        return self._sym

    def __repr__(self):
        return f"{type(self).__name__}(name={self.name!r}, value={self.value!r})"

    # arithmetic delegates to the symbol (`casadi_model.py:68-151`)
    def __add__(self, o):
        return sx.add(self._sym, _sym_of(o))

    def __radd__(self, o):
        return sx.add(_sym_of(o), self._sym)

    def __sub__(self, o):
        return sx.sub(self._sym, _sym_of(o))

    def __rsub__(self, o):
        return sx.sub(_sym_of(o), self._sym)

    def __mul__(self, o):
        return sx.mul(self._sym, _sym_of(o))

    def __rmul__(self, o):
        return sx.mul(_sym_of(o), self._sym)

    def __truediv__(self, o):
        return sx.div(self._sym, _sym_of(o))

    def __rtruediv__(self, o):
        return sx.div(_sym_of(o), self._sym)

    def __pow__(self, p, modulo=None):
        return sx.power(self._sym, _sym_of(p))

    def __rpow__(self, o):
        return sx.power(_sym_of(o), self._sym)

    def __abs__(self):
        return sx.fabs(self._sym)

    def __neg__(self):
        return sx.neg(self._sym)

    def __pos__(self):
        return self._sym

    def __lt__(self, o):
        return self._sym < _sym_of(o)

    def __le__(self, o):
        return self._sym <= _sym_of(o)

    def __gt__(self, o):
        return self._sym > _sym_of(o)

    def __ge__(self, o):
        return self._sym >= _sym_of(o)

    __hash__ = object.__hash__


class CasadiParameter(CasadiVariable):
    _causality = "parameter"


class CasadiInput(CasadiVariable):
    _causality = "input"

    @property
    def alg(self):
        raise AttributeError("Casadi Inputs should not have .alg assignments.")

    @alg.setter
    def alg(self, eq):
        raise ValueError(
            "Cannot assign algebraic equations to inputs. If this is for an MPC, try "
            "defining a constraint instead."
        )


class CasadiState(CasadiVariable):
    _causality = "local"

    def __init__(self, **kw):
        super().__init__(**kw)
        self._ode = None

    def fresh_copy(self):
        other = super().fresh_copy()
        other._ode = None
        return other

    @property
    def ode(self):
        return self._ode

    @ode.setter
    def ode(self, equation):
        self._ode = None if equation is None else sx.as_expr(_sym_of(equation))

    @property
    def alg(self):
        raise AttributeError("Casadi States should not have .alg assignments.")

    @alg.setter
    def alg(self, eq):
        raise AttributeError(
            "Casadi States should not have .alg assignments. If you need equality "
            "constraints in your MPC, please add them in the constraints."
        )


class CasadiOutput(CasadiVariable):
    _causality = "output"

    def __init__(self, **kw):
        super().__init__(**kw)
        self._alg = None

    def fresh_copy(self):
        other = super().fresh_copy()
        other._alg = None
        return other

    @property
    def alg(self):
        return self._alg

    @alg.setter
    def alg(self, equation):
        self._alg = None if equation is None else sx.as_expr(_sym_of(equation))


_GROUP_TYPES = {
    "inputs": CasadiInput,
    "outputs": CasadiOutput,
    "states": CasadiState,
    "parameters": CasadiParameter,
}


class CasadiModelConfig(pydantic.BaseModel):
    """Variable declaration container (`casadi_model.py:299-316`)."""

    model_config = ConfigDict(arbitrary_types_allowed=True, extra="allow")

    name: Optional[str] = None
    description: Optional[str] = None
    dt: float = 1.0
    inputs: List[Any] = Field(default_factory=list)
    outputs: List[Any] = Field(default_factory=list)
    states: List[Any] = Field(default_factory=list)
    parameters: List[Any] = Field(default_factory=list)


class CasadiModel:
    """Base class of symbolic models (`casadi_model.py:323-584`).

    Subclasses declare ``config: <ConfigClass>`` and implement
    ``setup_system()`` returning the objective.
    """

    config: CasadiModelConfig = CasadiModelConfig
    _forbidden_names = {"constraints", "cost_func", "time", "system", "integrator"}

    def __init__(self, **kwargs):
        object.__setattr__(self, "_is_initialized", False)
        cfg_cls = type(self).__annotations__.get("config", None)
        cfg_cls = self._resolve_config_class()
        overrides = {k: kwargs.pop(k) for k in list(kwargs) if k in _GROUP_TYPES}
        self.config = cfg_cls(**kwargs)
        self._vars: Dict[str, Dict[str, CasadiVariable]] = {}
        for group, vcls in _GROUP_TYPES.items():
            declared = [v.fresh_copy() if isinstance(v, CasadiVariable) else vcls(**v)
                        for v in getattr(self.config, group)]
            declared = {v.name: v for v in declared}
            for ov in overrides.get(group, []):
                ov = dict(ov) if isinstance(ov, dict) else {"name": ov.name, "value": ov.value}
                name = ov["name"]
                if name in declared:
                    declared[name].update(**ov)
                else:
                    declared[name] = vcls(**ov)
            self._vars[group] = declared
        bad = self._forbidden_names.intersection(self.variable_names())
        if bad:
            raise NameError(
                "The following variable names are not allowed as they intersect with "
                f"internal names of {type(self).__name__}: {' ,'.join(sorted(bad))}"
            )
        self.constraints = []
        self.time = sx.sym("time")
        object.__setattr__(self, "_is_initialized", True)
        objective = self.setup_system()
        self._assert_outputs_are_defined()
        from agentlib_mpc_amd.data_structures import objective as obj_mod

        if not hasattr(objective, "get_casadi_expression"):
            warnings.warn(
                "Model uses the deprecated objective formulation. Consider migrating to "
                "the new CombinedObjective formulation."
            )
            objective = obj_mod.CombinedObjective(
                obj_mod.SubObjective(expressions=sx.as_expr(_sym_of(objective)), name="objective")
            )
        self.objective = objective

    def _resolve_config_class(self):
        for klass in type(self).__mro__:
            # a config class assigned instead of annotated (``config = MyConfig``, e.g.
            # `tests/fixtures/casadi_test_model.py:62-63`) declares the variables as well
            c = klass.__dict__.get("config")
            if isinstance(c, type) and issubclass(c, CasadiModelConfig) and c is not CasadiModelConfig:
                return c
            ann = klass.__dict__.get("__annotations__", {})
            if "config" in ann:
                c = ann["config"]
                if isinstance(c, str):
                    import sys

                    mod = sys.modules[klass.__module__]
                    c = eval(c, vars(mod))  # annotation string from the model's module
                return c
        return CasadiModelConfig

    def setup_system(self):
        raise NotImplementedError("The ode is defined by the actual models inheriting from this class.")

    # -- variable access -------------------------------------------------------
    def variable_names(self):
        return [n for g in self._vars.values() for n in g]

    def __getattr__(self, item):
        vars_ = self.__dict__.get("_vars")
        if vars_ is not None:
            for group in vars_.values():
                if item in group:
                    return group[item]
        raise AttributeError(f"{type(self).__name__} has no attribute {item!r}")

    def __setattr__(self, key, value):
        if self.__dict__.get("_is_initialized") and key in self.variable_names():
            raise AttributeError(
                f"You are trying to create an instance attribute with the name {key}, "
                f"which is also in the variables of {type(self).__name__}. Assign "
                "equations via .alg for CasadiOutputs and .ode for CasadiStates."
            )
        object.__setattr__(self, key, value)

    def get(self, name: str) -> CasadiVariable:
        for group in self._vars.values():
            if name in group:
                return group[name]
        raise ValueError(f"Model {type(self).__name__} has no variable named {name!r}.")

    def _get_group(self, group, names):
        if names is None:
            return list(self._vars[group].values())
        missing = [n for n in names if n not in self._vars[group]]
        if missing:
            raise ValueError(f"Variables {missing} are not {group} of model {type(self).__name__}.")
        return [self._vars[group][n] for n in names]

    def get_states(self, names=None):
        return self._get_group("states", names)

    def get_inputs(self, names=None):
        return self._get_group("inputs", names)

    def get_outputs(self, names=None):
        return self._get_group("outputs", names)

    def get_parameters(self, names=None):
        return self._get_group("parameters", names)

    @property
    def inputs(self) -> List[CasadiInput]:
        return list(self._vars["inputs"].values())

    @property
    def outputs(self) -> List[CasadiOutput]:
        return list(self._vars["outputs"].values())

    @property
    def states(self) -> List[CasadiState]:
        return list(self._vars["states"].values())

    @property
    def parameters(self) -> List[CasadiParameter]:
        return list(self._vars["parameters"].values())

    @property
    def differentials(self) -> List[CasadiState]:
        return [s for s in self.states if s.ode is not None]

    @property
    def auxiliaries(self) -> List[CasadiState]:
        return [s for s in self.states if s.ode is None]

    @property
    def output_equations(self) -> List[sx.Expr]:
        """``y - alg(y)`` for every output (`casadi_model.py:489-493`)."""
        return [sx.sub(o.sym, o.alg) for o in self.outputs]

    def get_constraints(self) -> List[Tuple[sx.Expr, sx.Expr, sx.Expr]]:
        """User constraints followed by output equalities (`casadi_model.py:458-467`)."""
        base = [(sx.as_expr(_sym_of(lb)), sx.as_expr(_sym_of(f)), sx.as_expr(_sym_of(ub)))
                for lb, f, ub in self.constraints]
        eq = [(sx.ZERO, alg, sx.ZERO) for alg in self.output_equations]
        return base + eq

    def _assert_outputs_are_defined(self):
        for out in self.outputs:
            if out.alg is None:
                raise ValueError(
                    f"Output '{out.name}' was not initialized with an equation. Make sure "
                    f"you specify '{out.name}.alg' in 'setup_system()'."
                )

    # -- objective helpers (`casadi_model.py:516-545`) ---------------------------
    def create_sub_objective(self, expressions, weight=1, name: str = None):
        from agentlib_mpc_amd.data_structures.objective import SubObjective

        return SubObjective(expressions=expressions, weight=weight, name=name)

    def create_change_penalty(self, expressions, weight=1, name: str = None):
        from agentlib_mpc_amd.data_structures.objective import ChangePenaltyObjective

        return ChangePenaltyObjective(expressions=expressions, weight=weight, name=name)

    def create_combined_objective(self, *objectives, normalization: float = 1.0):
        from agentlib_mpc_amd.data_structures.objective import CombinedObjective

        return CombinedObjective(*objectives, normalization=normalization)

    def create_conditional_objective(self, *condition_objective_pairs, default_objective=None):
        """`casadi_model.py:549-557`."""
        from agentlib_mpc_amd.data_structures.objective import ConditionalObjective

        return ConditionalObjective(*condition_objective_pairs, default_objective=default_objective)
