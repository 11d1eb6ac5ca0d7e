"""Objective containers (symbolic part).

Mirrors the reference's objective API (`agentlib_mpc/data_structures/objective.py`):
``SubObjective`` (:74-237), ``ChangePenaltyObjective`` (:239-296),
``CombinedObjective`` (:297-453), ``ConditionalObjective`` (:456-621) and
``CompositeWeight`` (:10-71): the symbolic side that builds the NLP and the
post-hoc evaluation ``calculate_values`` that the backends write into the stats
file (``obj_<name>`` columns, `core/casadi_backend.py:291-323`).

Evaluation: the reference re-parses the ``str()`` of a CasADi expression with
``eval`` and, when the string contains ``sq(``, evaluates it with every ``sq(``
read as ``(`` and squares the whole term (:166-224) -- for a term that mixes a
square with other operations that is not the term's value.  The traced
expression is evaluated numerically on the result grid with the same rule
(``REFERENCE_SQ_RULE = True``, so the ``obj_<name>`` stats columns equal the
reference's); set it to False for the term's mathematical value.
"""

from __future__ import annotations

import warnings
from typing import Union

import numpy as np
import pandas as pd

from agentlib_mpc_amd import symbolic as sx


#: evaluate a term containing sq() the reference's way (squares removed, whole term squared)
REFERENCE_SQ_RULE = True


def _column(df, name):
    for kind in ("variable", "parameter"):
        if (kind, name) in df.columns:
            return df.loc[:, (kind, name)].to_numpy(dtype=float)
    return None


def _evaluate_on(df, expr, drop_last=True):
    """Values of a traced expression on the rows of a result frame (``time`` = index)."""
    e = expr.sym if hasattr(expr, "sym") else sx.as_expr(expr)
    vals = {}
    for s in sx.free_symbols([e]):
        col = df.index.to_numpy(dtype=float) if s.name == "time" else _column(df, s.name)
        if col is None:
            raise KeyError(s.name)
        vals[s] = col[:-1] if drop_last else col
    n = len(df) - 1 if drop_last else len(df)
    return np.broadcast_to(np.asarray(sx.evaluate([e], vals)[0], float), (max(n, 0),))


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

    def evaluate(self, df):
        """Weight values on the frame rows (`objective.py:63-71`)."""
        result = self.constant_factor
        for name in self.param_names:
            result = result * df.loc[:, ("parameter", name)]
        return result if isinstance(result, pd.Series) else pd.Series(result, index=df.index)

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

    _warned_names = set()

    def calculate_value(self, data, weight):
        """Rectangle rule over the result grid (`objective.py:135-139`)."""
        ts = np.diff(data.index.to_numpy(dtype=float))
        try:
            expr = self.expression.sym if hasattr(self.expression, "sym") else self.expression
            squared = False
            if REFERENCE_SQ_RULE:
                expr, squared = sx.strip_squares(expr)
            result = _evaluate_on(data, expr)
            if squared:
                result = result ** 2
        except KeyError:
            if self.name not in SubObjective._warned_names:
                warnings.warn(f"Unable to evaluate expression {self.name}. Some terms will be ignored when "
                              "displaying the objective value. The control still works, only the objective "
                              "logging is affected.", RuntimeWarning)
                SubObjective._warned_names.add(self.name)
            return 0
        return float(np.sum(np.asarray(weight, float) * result * ts))


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

    def calculate_value(self, series, weight):
        """``w**2 * (u_k - u_{k-1})**2 * ts`` summed (`objective.py:288-294`)."""
        diff = series.diff().to_numpy(dtype=float)[1:]
        ts = np.diff(series.index.to_numpy(dtype=float))
        res = pd.Series(np.asarray(weight, float) ** 2 * diff ** 2 * ts)
        return float(res.dropna().sum())


def _weight_values(weight, df, change_penalty: bool):
    """Numeric weight of a term on the frame rows (`objective.py:366-386`)."""
    from agentlib_mpc_amd.models.casadi_model import CasadiParameter

    if isinstance(weight, CasadiParameter):
        col = df.loc[:, ("parameter", weight.name)]
    elif isinstance(weight, CompositeWeight):
        col = weight.evaluate(df)
    else:
        return weight
    return col.shift(-1).iloc[:-1].to_numpy(dtype=float) if change_penalty else col.iloc[:-1].to_numpy(dtype=float)


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

    # -- post-hoc evaluation (`objective.py:342-453`) -------------------------------
    def calculate_values(self, result_df, grid):
        """Value of every term (and ``total``) on ``grid`` from a ``Results.df``."""
        values = {}
        df = self._prepare_dataframe(result_df, grid)
        total = 0.0
        if grid is not None:
            start = result_df.index.get_loc(grid[0])
            helper_grid = np.insert(np.asarray(grid, float), 0, result_df.index[start - 1]) if start > 0 else grid
            df_helper = self._prepare_dataframe(result_df, helper_grid)
        else:
            df_helper = self._prepare_dataframe(result_df, grid)
        for obj in self.objectives:
            if isinstance(obj, ChangePenaltyObjective):
                weight = _weight_values(obj.weight, df_helper, True)
                val = obj.calculate_value(df_helper.loc[:, ("variable", obj.get_control_name())], weight)
            else:
                val = obj.calculate_value(df, _weight_values(obj.weight, df, False))
            values[obj.name] = val / self.normalization
            if values[obj.name] is not None:
                total += values[obj.name]
        values["total"] = total
        return values

    def _prepare_dataframe(self, df, grid=None):
        """Parameters forward-filled, collocation-only variables filled from the following
        collocation points, rows restricted to ``grid`` (`objective.py:397-453`)."""
        new_df = df.copy()
        for col in new_df.columns:
            if col[0] == "parameter":
                new_df[col] = new_df[col].ffill()
            elif col[0] == "variable" and grid is not None and len(grid) > 0:
                on_grid = [v for v in grid if v in new_df.index]
                if new_df.loc[on_grid, col].isna().all():
                    new_df[col] = _fill_collocation_nans(new_df[col])
        if grid is not None and len(grid) > 0:
            valid = [g for g in grid if g in new_df.index]
            if valid:
                new_df = new_df.loc[valid]
        return new_df


def _fill_collocation_nans(series):
    """Each NaN takes the mean of the run of values that follows it (`objective.py:438-453`)."""
    vals = series.to_numpy(dtype=float)
    out = vals.copy()
    for i in np.flatnonzero(np.isnan(vals)):
        j = i + 1
        while j < len(vals) and not np.isnan(vals[j]):
            j += 1
        if j > i + 1:
            out[i] = vals[i + 1:j].mean()
    return pd.Series(out, index=series.index)


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

    def calculate_values(self, result_df, grid):
        """Each objective evaluated on the rows where its condition holds
        (`objective.py:501-525`)."""
        df = self.default_objective._prepare_dataframe(result_df.copy(), grid)
        masks = {id(self.default_objective): np.ones(len(df), bool)}
        objs = {id(self.default_objective): self.default_objective}
        for cond, objective in self.condition_objective_pairs:
            m = self._evaluate_condition(cond, df)
            masks[id(objective)] = m
            objs[id(objective)] = objective
            masks[id(self.default_objective)] &= ~m
        values, total = {}, 0.0
        for k, objective in objs.items():
            sub = df.loc[masks[k]].copy()
            if len(sub) == 0:
                continue
            for name, v in objective.calculate_values(sub, None).items():
                if name == "total":
                    continue
                values[name] = values.get(name, 0) + v
                if v is not None:
                    total += v
        values["total"] = total
        return values

    @staticmethod
    def _evaluate_condition(condition, df):
        try:
            return np.asarray(_evaluate_on(df, condition, drop_last=False), float) != 0.0
        except KeyError:
            return np.zeros(len(df), bool)
