"""Optimization variable groups and systems.

Restates the reference's variable-group layer:
``OptimizationVariable.declare`` / ``OptimizationParameter.declare``
(`optimization_backends/casadi_/core/VariableGroup.py:39-137`, `148-223`),
``System`` (`core/system.py:16-74`), ``BaseSystem``
(`casadi_/basic.py:29-101`), ``FullSystem`` (`casadi_/full.py:18-33`) and
``CasadiADMMSystem`` (`casadi_/admm.py:23-116`).  Group declaration order is
significant: it defines the result column order (`core/discretization.py:455-481`).
"""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Sequence, Tuple

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.data_structures.mpc_datamodels import VariableReference
from agentlib_mpc_amd.data_structures.objective import CombinedObjective, SubObjective
from agentlib_mpc_amd.models.casadi_model import CasadiInput, CasadiModel, CasadiParameter


def _check_ref_in_full(ref: Sequence[str], full: Sequence[str]):
    diff = set(ref).difference(full)
    if diff:
        raise ValueError(
            "The variables from the variable ref are not a subset of the model "
            f"variables. The following variables are wrong: {diff}"
        )


@dataclasses.dataclass(frozen=True, eq=False)
class OptimizationQuantity:
    name: str
    full_symbolic: Tuple[sx.Expr, ...]
    dim: int
    ref_names: Tuple[str, ...]
    full_names: Tuple[str, ...]
    use_in_stage_function: bool

    def __hash__(self):
        return hash(self.name)


@dataclasses.dataclass(frozen=True, eq=False)
class OptimizationVariable(OptimizationQuantity):
    #: bounds used for entries that are not supplied at runtime (model lb/ub)
    default_lb: Tuple[float, ...] = ()
    default_ub: Tuple[float, ...] = ()
    binary: bool = False

    @classmethod
    def declare(cls, denotation: str, variables, ref_list: Sequence[str],
                use_in_stage_function: bool = True, assert_complete: bool = False,
                binary: bool = False) -> "OptimizationVariable":
        full_sym, full_names, ref_ordered, lbs, ubs = [], [], [], [], []
        for var in variables:
            if assert_complete and var.name not in ref_list:
                raise ValueError(f"The variable {var.name} which is defined in the model "
                                 f" has to be defined in the ModuleConfig!")
            full_sym.append(var.sym)
            full_names.append(var.name)
            if var.name in ref_list:
                ref_ordered.append(var.name)
                lbs.append(math.nan)   # supplied at runtime
                ubs.append(math.nan)
            else:
                lbs.append(float(var.lb))
                ubs.append(float(var.ub))
        _check_ref_in_full(ref_list, full_names)
        return cls(name=denotation, full_symbolic=tuple(full_sym), dim=len(full_sym),
                   ref_names=tuple(ref_ordered), full_names=tuple(full_names),
                   use_in_stage_function=use_in_stage_function,
                   default_lb=tuple(lbs), default_ub=tuple(ubs), binary=binary)


@dataclasses.dataclass(frozen=True, eq=False)
class OptimizationParameter(OptimizationQuantity):
    #: default values for entries not supplied at runtime (model value)
    defaults: Tuple[float, ...] = ()

    @classmethod
    def declare(cls, denotation: str, variables, ref_list: Sequence[str],
                use_in_stage_function: bool = True,
                assert_complete: bool = False) -> "OptimizationParameter":
        full_sym, full_names, ref_ordered, defaults = [], [], [], []
        for var in variables:
            if assert_complete and var.name not in ref_list:
                raise AssertionError(f"The variable {var.name} which is defined in the model "
                                     f" has to be defined in the ModuleConfig!")
            full_sym.append(var.sym)
            full_names.append(var.name)
            if var.name in ref_list:
                ref_ordered.append(var.name)
                defaults.append(math.nan)
            else:
                if var.value is None:
                    raise ValueError(
                        f"Parameter '{var.name}' is not declared in the module config. "
                        "Tried using default from model  but it was 'None'."
                    )
                defaults.append(float(var.value))
        _check_ref_in_full(ref_list, full_names)
        return cls(name=denotation, full_symbolic=tuple(full_sym), dim=len(full_sym),
                   ref_names=tuple(ref_ordered), full_names=tuple(full_names),
                   use_in_stage_function=use_in_stage_function, defaults=tuple(defaults))


class System:
    """Holds variable groups; iteration order = attribute insertion order."""

    def initialize(self, model: CasadiModel, var_ref: VariableReference):
        raise NotImplementedError

    @property
    def variables(self) -> List[OptimizationVariable]:
        return [v for v in self.__dict__.values() if isinstance(v, OptimizationVariable)]

    @property
    def parameters(self) -> List[OptimizationParameter]:
        return [v for v in self.__dict__.values() if isinstance(v, OptimizationParameter)]

    @property
    def quantities(self):
        return self.variables + self.parameters


class BaseSystem(System):
    """`casadi_/basic.py:29-101`."""

    def initialize(self, model: CasadiModel, var_ref: VariableReference):
        self.states = OptimizationVariable.declare("state", model.get_states(var_ref.states),
                                                   var_ref.states, assert_complete=True)
        self.controls = OptimizationVariable.declare("control", model.get_inputs(var_ref.controls),
                                                     var_ref.controls, assert_complete=True)
        self.algebraics = OptimizationVariable.declare("z", model.auxiliaries, [])
        self.outputs = OptimizationVariable.declare("y", model.outputs, var_ref.outputs)
        self.non_controlled_inputs = OptimizationParameter.declare(
            "d", model.get_inputs(var_ref.inputs), var_ref.inputs, assert_complete=True)
        self.model_parameters = OptimizationParameter.declare(
            "parameter", model.parameters, var_ref.parameters)
        self.initial_state = OptimizationParameter.declare(
            "initial_state", model.get_states(var_ref.states), var_ref.states,
            use_in_stage_function=False, assert_complete=True)
        states = model.get_states(var_ref.states)
        missing_ode = [s.name for s in states if s.ode is None]
        if missing_ode:
            raise ValueError(f"States {missing_ode} are declared as MPC states but have no ode.")
        self.ode = [s.ode for s in states]
        self.objective: CombinedObjective = model.objective
        self.model_constraints = model.get_constraints()
        self.time = model.time


class FullSystem(BaseSystem):
    """`casadi_/full.py:18-33`: adds the previous control ``u_prev``."""

    def initialize(self, model: CasadiModel, var_ref: VariableReference):
        super().initialize(model, var_ref)
        self.last_control = OptimizationParameter.declare(
            "u_prev", model.get_inputs(var_ref.controls), var_ref.controls,
            use_in_stage_function=False, assert_complete=True)


class ADMMSystem(FullSystem):
    """`casadi_/admm.py:23-116`: coupling/exchange groups and ADMM terms."""

    def initialize(self, model: CasadiModel, var_ref: adt.VariableReference):
        super().initialize(model, var_ref)
        coup_names = [c.name for c in var_ref.couplings]
        exch_names = [c.name for c in var_ref.exchange]
        pure_outs = [o for o in model.outputs if o.name not in coup_names + exch_names]
        # re-declaring keeps the dict position of "outputs" (insertion order)
        self.outputs = OptimizationVariable.declare("y", pure_outs, var_ref.outputs)
        self.local_couplings = OptimizationVariable.declare(
            "local_couplings", [model.get(n) for n in coup_names], coup_names)
        means = [c.mean for c in var_ref.couplings]
        self.global_couplings = OptimizationParameter.declare(
            "global_couplings", [CasadiInput(name=n) for n in means], means)
        mults = [c.multiplier for c in var_ref.couplings]
        self.multipliers = OptimizationParameter.declare(
            "multipliers", [CasadiInput(name=n) for n in mults], mults)
        self.local_exchange = OptimizationVariable.declare(
            "local_exchange", [model.get(n) for n in exch_names], exch_names)
        diffs = [c.mean_diff for c in var_ref.exchange]
        self.exchange_diff = OptimizationParameter.declare(
            "average_diff", [CasadiInput(name=n) for n in diffs], diffs)
        emults = [c.multiplier for c in var_ref.exchange]
        self.exchange_multipliers = OptimizationParameter.declare(
            "exchange_multipliers", [CasadiInput(name=n) for n in emults], emults)
        self.penalty_factor = OptimizationParameter.declare(
            "rho", [CasadiParameter(name="penalty_factor")], ["penalty_factor"])

        rho = self.penalty_factor.full_symbolic[0]
        terms = []
        for i in range(len(var_ref.couplings)):
            z_bar = self.global_couplings.full_symbolic[i]
            x_loc = self.local_couplings.full_symbolic[i]
            lam = self.multipliers.full_symbolic[i]
            terms.append(lam * x_loc)
            terms.append(rho / 2 * (z_bar - x_loc) ** 2)
        for i in range(len(var_ref.exchange)):
            diff = self.exchange_diff.full_symbolic[i]
            x_loc = self.local_exchange.full_symbolic[i]
            lam = self.exchange_multipliers.full_symbolic[i]
            terms.append(lam * x_loc)
            terms.append(rho / 2 * (diff - x_loc) ** 2)
        from agentlib_mpc_amd.data_structures.objective import ConditionalObjective

        if isinstance(self.objective, ConditionalObjective):
            # the reference's in-place append (`admm.py:90-116`) fails on the read-only
            # ``objectives`` property of a ConditionalObjective as well
            raise NotImplementedError("ADMM terms cannot be added to a ConditionalObjective")
        # the reference appends to the model's objective list in place
        self.objective = CombinedObjective(
            *self.objective.objectives,
            *[SubObjective(t, name="admm_augmentation_term") for t in terms],
            normalization=self.objective.normalization,
        )
