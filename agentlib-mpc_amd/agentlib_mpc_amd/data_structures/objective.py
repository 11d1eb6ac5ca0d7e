"""Objective containers (symbolic part).

Mirrors the reference's objective API (`agentlib_mpc/data_structures/objective.py`):
``SubObjective`` (:74-133), ``ChangePenaltyObjective`` (:238-296),
``CombinedObjective`` (:299-340) and ``CompositeWeight`` (:10-71).  Only the
symbolic side used to build the NLP is implemented; the post-hoc pandas
evaluation (``calculate_values``, :342-395) is reporting and out of scope.
"""

from __future__ import annotations

from typing import Union

from agentlib_mpc_amd import symbolic as sx


def _weight_sym(w):
    if isinstance(w, CompositeWeight):
        return w.sym
    if hasattr(w, "sym"):
        return w.sym
    return w


class CompositeWeight:
    """Product of parameters and constants used as an objective weight
    (`objective.py:10-71`)."""

    def __init__(self, base_component):
        from agentlib_mpc_amd.models.casadi_model import CasadiParameter

        self.param_names = []
        self.constant_factor = 1.0
        if isinstance(base_component, CasadiParameter):
            self.param_names = [base_component.name]
            self.sym = base_component.sym
        elif isinstance(base_component, (int, float)):
            self.constant_factor = float(base_component)
            self.sym = base_component
        elif isinstance(base_component, CompositeWeight):
            self.param_names = list(base_component.param_names)
            self.constant_factor = base_component.constant_factor
            self.sym = base_component.sym

    def multiply_by(self, other):
        from agentlib_mpc_amd.models.casadi_model import CasadiParameter

        if isinstance(other, CasadiParameter):
            self.param_names.append(other.name)
            self.sym = self.sym * other.sym
        elif isinstance(other, (int, float)):
            self.constant_factor *= other
            self.sym = self.sym * other
        elif isinstance(other, CompositeWeight):
            self.param_names.extend(other.param_names)
            self.constant_factor *= other.constant_factor
            self.sym = self.sym * other.sym
        return self


class SubObjective:
    """One weighted objective term (`objective.py:74-133`)."""

    def __init__(self, expressions, weight: Union[float, int, object] = 1, name: str = None):
        self.expression = expressions
        self.weight = weight
        self.name = name or f"obj_{id(self)}"

    def __add__(self, other):
        if isinstance(other, SubObjective):
            return CombinedObjective(self, other)
        raise TypeError(f"Cannot add SubObjective with {type(other)}")

    def __mul__(self, other):
        return SubObjective(self.expression, _multiply_weights(self.weight, other), f"scaled_{self.name}")

    def get_weighted_expression(self):
        expr = self.expression.sym if hasattr(self.expression, "sym") else self.expression
        return sx.mul(_weight_sym(self.weight), expr)


class ChangePenaltyObjective(SubObjective):
    """Δu penalty on a control (`objective.py:238-296`); realised in the
    discretisation as ``w**2 * (u_k - u_{k-1})**2`` (`core/delta_u.py:13-26`)."""

    def __init__(self, expressions, weight=1, name: str = None):
        from agentlib_mpc_amd.models.casadi_model import CasadiInput

        if not isinstance(expressions, CasadiInput):
            raise TypeError(
                "Tried to create a control change objective with an expression or "
                "different type of CasadiVariable. Currently, only raw CasadiInputs "
                "are supported."
            )
        self.control = expressions
        super().__init__(expressions=expressions, weight=weight, name=name or f"delta_{expressions.name}")

    def __mul__(self, mul):
        return ChangePenaltyObjective(self.control, _multiply_weights(self.weight, mul), f"scaled_{self.name}")

    def get_control_name(self):
        return self.control.name

    def get_weighted_expression(self):
        return sx.ZERO


def _multiply_weights(w1, w2):
    from agentlib_mpc_amd.models.casadi_model import CasadiParameter

    if isinstance(w1, (int, float)) and isinstance(w2, (int, float)):
        return w1 * w2
    if isinstance(w1, (CasadiParameter, CompositeWeight)) or isinstance(w2, (CasadiParameter, CompositeWeight)):
        res = CompositeWeight(w1)
        res.multiply_by(w2)
        return res
    return _weight_sym(w1) * _weight_sym(w2)


class CombinedObjective:
    """Sum of objective terms over a normalisation (`objective.py:299-340`)."""

    def __init__(self, *objectives, normalization: float = 1.0):
        self.objectives = list(objectives)
        self.normalization = normalization

    def __add__(self, other):
        if isinstance(other, CombinedObjective):
            return CombinedObjective(*self.objectives, *other.objectives, normalization=self.normalization)
        raise TypeError(f"Cannot add CombinedObjective with {type(other)}")

    def __mul__(self, other):
        return CombinedObjective(*[o * other for o in self.objectives], normalization=self.normalization)

    def get_delta_u_objectives(self):
        return [o for o in self.objectives if isinstance(o, ChangePenaltyObjective)]

    def get_casadi_expression(self):
        total = sx.ZERO
        for obj in self.objectives:
            total = sx.add(total, obj.get_weighted_expression())
        return sx.div(total, self.normalization)


class ConditionalObjective:
    """Switches between objectives by conditions (`objective.py:456-499`):
    ``if_else(c_1, o_1, if_else(c_2, o_2, ... default))``; the conditions are
    expressions of the model variables (non-differentiable switches, as in CasADi)."""

    def __init__(self, *condition_objective_pairs, default_objective=None):
        self.condition_objective_pairs = condition_objective_pairs
        self.default_objective = default_objective or CombinedObjective()
        self.all_objectives = [self.default_objective]
        for _, objective in condition_objective_pairs:
            if objective not in self.all_objectives:
                self.all_objectives.append(objective)
        self._flattened_objectives = []
        for obj in self.all_objectives:
            if hasattr(obj, "objectives"):
                self._flattened_objectives.extend(obj.objectives)

    @property
    def objectives(self):
        return self._flattened_objectives

    @property
    def normalization(self):
        return 1.0

    def get_casadi_expression(self):
        result = self.default_objective.get_casadi_expression()
        for condition, objective in reversed(self.condition_objective_pairs):
            cond = condition.sym if hasattr(condition, "sym") else condition
            result = sx.if_else(sx.as_expr(cond), objective.get_casadi_expression(), result)
        return result

    def get_delta_u_objectives(self):
        out = []
        for objective in self.all_objectives:
            for d in objective.get_delta_u_objectives():
                if d not in out:
                    out.append(d)
        return out
