"""MPC data models shared by the backend and its callers.

Mirrors `agentlib_mpc/data_structures/mpc_datamodels.py` (variable references
:53-93, ``MPCVariable`` :96-108, ``DiscretizationOptions`` :29-46,
``stats_path`` :114-116), `agentlib_mpc/data_structures/interpolation.py:6-27`
and the discretisation enums / options of
`agentlib_mpc/data_structures/casadi_utils.py:42-81`.
"""

from __future__ import annotations

import dataclasses
import math
from enum import Enum
from itertools import chain
from pathlib import Path
from typing import Any, List, Union

import pydantic
from pydantic import ConfigDict, Field


class InterpolationMethods(str, Enum):
    linear = "linear"
    previous = "previous"
    no_interpolation = "no_interpolation"
    spline3 = "spline3"
    mean_over_interval = "mean_over_interval"


class DiscretizationMethod(str, Enum):
    collocation = "collocation"
    multiple_shooting = "multiple_shooting"


class CollocationMethod(str, Enum):
    radau = "radau"
    legendre = "legendre"


class Integrators(str, Enum):
    cvodes = "cvodes"
    rk = "rk"
    euler = "euler"


class Solvers(str, Enum):
    ipopt = "ipopt"
    fatrop = "fatrop"
    sqpmethod = "sqpmethod"
    qpoases = "qpoases"
    gurobi = "gurobi"
    bonmin = "bonmin"
    proxqp = "proxqp"
    osqp = "osqp"


class DiscretizationOptions(pydantic.BaseModel):
    model_config = ConfigDict(extra="allow")
    time_step: float = Field(default=60, ge=0)
    prediction_horizon: int = Field(default=5, ge=0)


class CasadiDiscretizationOptions(DiscretizationOptions):
    model_config = ConfigDict(extra="forbid")
    method: DiscretizationMethod = DiscretizationMethod.collocation
    collocation_order: int = Field(default=3, ge=1, le=9)
    collocation_method: CollocationMethod = CollocationMethod.legendre
    integrator: Integrators = Integrators.cvodes


class SolverOptions(pydantic.BaseModel):
    """``solver`` block of the backend config (`casadi_utils.py:78-81`).

    ``name`` is kept for config compatibility; every name is served by the
    MI355X interior-point kernel.  IPOPT-style options are read from
    ``options["ipopt"]`` / ``options["ipopt.<key>"]``.
    """

    model_config = ConfigDict(extra="forbid")
    name: Solvers = Solvers.ipopt
    options: dict = Field(default_factory=dict)


@dataclasses.dataclass
class BaseVariableReference:
    def all_variables(self) -> List[str]:
        return list(chain.from_iterable(self.__dict__.values()))

    def __contains__(self, item):
        return item in set(self.all_variables())


@dataclasses.dataclass
class VariableReference(BaseVariableReference):
    states: List[str] = dataclasses.field(default_factory=list)
    controls: List[str] = dataclasses.field(default_factory=list)
    inputs: List[str] = dataclasses.field(default_factory=list)
    parameters: List[str] = dataclasses.field(default_factory=list)
    outputs: List[str] = dataclasses.field(default_factory=list)


class MPCVariable:
    """Minimal stand-in for agentlib's ``AgentVariable`` + interpolation method.

    Any object with ``name``, ``value``, ``lb``, ``ub`` and
    ``interpolation_method`` attributes (e.g. the reference's ``MPCVariable``)
    is accepted by :meth:`solve`.
    """

    def __init__(self, name: str, value: Any = None, lb: Any = -math.inf, ub: Any = math.inf,
                 interpolation_method: Union[str, InterpolationMethods] = InterpolationMethods.linear,
                 alias: str = None, source: Any = None, **extra):
        self.name = name
        self.value = value
        self.lb = lb
        self.ub = ub
        self.interpolation_method = InterpolationMethods(interpolation_method)
        self.alias = alias or name
        self.source = source
        self.extra = extra

    def __repr__(self):
        return f"MPCVariable(name={self.name!r}, value={self.value!r}, lb={self.lb!r}, ub={self.ub!r})"


def stats_path(path: Union[Path, str]) -> Path:
    res_file = Path(path)
    return Path(res_file.parent, "stats_" + res_file.name)
