"""Data-driven (NARX) models: ``CasadiMLModel``.

Restates `agentlib_mpc/models/casadi_ml_model.py`:

* ``CasadiMLModelConfig`` (:45-137): ``ml_model_sources`` (serialized models or
  paths; duplicate outputs and unknown inputs/outputs are configuration
  errors) and ``dt`` (overridden by the models' common ``dt``).
* ``CasadiMLModel.__init__`` (:160-180): registers one predictor per output
  (``register_ml_models`` :327-354), the lag table ``lags_dict`` / ``max_lag``
  (:230-243, the maximum lag of every feature over all models), symbols for
  lagged values ``lags_mx_store`` (:245-252, named ``name_with_lag``), and
  algebraic equations for non-recursive model outputs
  (``_fill_algebraic_equations_with_bb_output`` :356-375).
* ``make_predict_function_for_mpc`` (:458-462) → here :meth:`predict_step`:
  next values of the recursive (state) outputs, ``difference`` outputs added
  to the current value (``_evaluate_bb_models_symbolically`` :377-420).
  White-box differentials inside an ML model would need the reference's
  cvodes/idas integrators (:272-325), which are not on the MI355X path: such
  models raise ``NotImplementedError``.
* ``auxiliaries`` (:637-648): states with neither an ode nor an ML model.

Simulation (``do_step``, past-value bookkeeping) belongs to the agentlib
runtime and is out of scope.
"""

from __future__ import annotations

import logging
from itertools import chain
from pathlib import Path
from typing import Dict, List, Union

from pydantic import Field, field_validator, model_validator

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.data_structures import ml_model_datatypes as mlt
from agentlib_mpc_amd.data_structures.ml_model_datatypes import OutputType, name_with_lag
from agentlib_mpc_amd.models.casadi_model import CasadiModel, CasadiModelConfig, CasadiState
from agentlib_mpc_amd.models.casadi_predictor import CasadiANN, CasadiPredictor
from agentlib_mpc_amd.models.serialized_ml_model import SerializedMLModel

logger = logging.getLogger(__name__)


def compute_dupes(collection) -> list:
    dupes, seen = [], set()
    for element in collection:
        if element in seen:
            dupes.append(element)
        else:
            seen.add(element)
    return dupes


def _names(group) -> List[str]:
    return [v.name if hasattr(v, "name") else v["name"] for v in group]


class CasadiMLModelConfig(CasadiModelConfig):
    ml_model_sources: List[Union[SerializedMLModel, Path, str, dict]] = Field(default_factory=list)
    dt: Union[float, int] = Field(default=1, validate_default=True)

    @field_validator("ml_model_sources", mode="before")
    @classmethod
    def check_or_load_models(cls, sources, info):
        loaded = []
        for src in sources:
            if not isinstance(src, SerializedMLModel):
                src = SerializedMLModel.load_serialized_model(src)
            loaded.append(src)
        outputs = _names(info.data.get("outputs", []))
        for s in loaded:
            for out_name, feat in s.output.items():
                if out_name in outputs and feat.recursive:
                    raise ValueError(
                        f"Provided ML-model defines recursive output {out_name}, however in the model "
                        "config it is listed under 'outputs'. A recursive model output can only be "
                        "associated with a 'state'.")
        if len({s.dt for s in loaded}) > 1:
            raise ValueError(f"Provided MLModel's need to have the same 'dt'. Provided dt are "
                             f"{ {s.dt for s in loaded} }")
        all_outputs = list(chain.from_iterable(s.output.keys() for s in loaded))
        all_inputs = list(chain.from_iterable(s.input.keys() for s in loaded))
        out_names = _names(info.data.get("states", [])) + outputs
        in_names = _names(info.data.get("inputs", [])) + _names(info.data.get("states", []))
        dupes = compute_dupes(all_outputs)
        if dupes:
            raise ValueError(f"The MLModel's that were provided define the same output multiple "
                             f"times. Duplicates are: {dupes}")
        bad_in = set(all_inputs) - set(in_names)
        bad_out = set(all_outputs) - set(out_names)
        if bad_in:
            raise ValueError(f"Inputs specified by MLModels do not appear in model: {bad_in}")
        if bad_out:
            raise ValueError(f"Outputs specified by MLModels do not appear in model states / outputs: {bad_out}")
        return loaded

    @model_validator(mode="after")
    def check_dt(self):
        if self.ml_model_sources:
            ml_dt = self.ml_model_sources[0].dt
            if self.dt != ml_dt:
                logger.warning("Time step (dt) of model and supplied MLModels does not match. "
                               "Setting the model time step to %s.", ml_dt)
                self.dt = ml_dt
        return self


class CasadiMLModel(CasadiModel):
    """Model whose states/outputs are (partly) predicted by serialized ML models."""

    config: CasadiMLModelConfig

    def __init__(self, **kwargs):
        object.__setattr__(self, "_ml_ready", False)
        super().__init__(**kwargs)
        self.ml_model_dict, self.casadi_ml_model_dict = self.register_ml_models()
        self.lags_dict, self.max_lag = self._create_lags_dict()
        self.lags_mx_store = self._create_lags_mx_variables()
        self._fill_algebraic_equations_with_bb_output()
        object.__setattr__(self, "_ml_ready", True)
        self._assert_outputs_are_defined()
        if self.differentials:
            raise NotImplementedError(
                "white-box differential states inside a CasadiMLModel need the reference's cvodes/idas "
                "integrators, which are not part of the MI355X backend")

    def setup_system(self):
        return 0

    @property
    def dt(self):
        return self.config.dt

    # -- registration (`casadi_ml_model.py:327-375`) ---------------------------------
    def register_ml_models(self):
        by_outputs = {tuple(m.output.keys()): m for m in self.config.ml_model_sources}
        ml_model_dict: Dict[str, SerializedMLModel] = {}
        casadi_dict: Dict[str, CasadiANN] = {}
        for var in self.outputs + self.states:
            for names, m in by_outputs.items():
                if var.name in names:
                    casadi_dict[var.name] = CasadiPredictor.from_serialized_model(m)
                    ml_model_dict[var.name] = m
        return ml_model_dict, casadi_dict

    def _create_lags_dict(self):
        lags: Dict[str, int] = {}
        for m in self.config.ml_model_sources:
            for name, feat in {**m.input, **m.output}.items():
                cur = lags.setdefault(name, 1)
                if feat.lag > cur:
                    lags[name] = feat.lag
        return lags, (max(lags.values()) if lags else 1)

    def _create_lags_mx_variables(self) -> Dict[str, sx.Expr]:
        store = {}
        for name, max_lag in self.lags_dict.items():
            for lag in range(1, max_lag):
                l_name = name_with_lag(name, lag)
                store[l_name] = sx.sym(l_name)
        return store

    def _get_lagged_symbolic(self, name: str) -> sx.Expr:
        try:
            return self.get(name).sym
        except ValueError:
            return self.lags_mx_store[name]

    def _fill_algebraic_equations_with_bb_output(self):
        for var_name, m in self.ml_model_dict.items():
            if m.output[var_name].recursive:
                continue
            if self.get(var_name).alg is not None:
                raise RuntimeError(f"output {var_name} has both an equation and an ML model")
            cols = mlt.column_order(inputs=m.input, outputs=m.output)
            x = [self._get_lagged_symbolic(n) for n in cols]
            idx = list(m.output).index(var_name)
            self.get(var_name).alg = self.casadi_ml_model_dict[var_name].predict(x)[idx]

    # -- prediction (`casadi_ml_model.py:377-420`, `:458-462`) -----------------------
    def predict_step(self) -> Dict[str, sx.Expr]:
        """Next value of every recursive ML output, in the model's own symbols
        (current values = variable symbols, lagged values = ``lags_mx_store``)."""
        out: Dict[str, sx.Expr] = {}
        for name, m in self.ml_model_dict.items():
            if not m.output[name].recursive:
                continue
            cols = mlt.column_order(inputs=m.input, outputs=m.output)
            x = [self._get_lagged_symbolic(n) for n in cols]
            idx = list(m.output).index(name)
            res = self.casadi_ml_model_dict[name].predict(x)[idx]
            if m.output[name].output_type == OutputType.difference:
                res = sx.add(res, self._get_lagged_symbolic(name))
            out[name] = res
        return out

    @property
    def bb_states(self) -> List[CasadiState]:
        return [v for v in self.states if v.name in self.ml_model_dict]

    @property
    def auxiliaries(self) -> List[CasadiState]:
        return [v for v in self.states if v.ode is None and v.name not in self.__dict__.get("ml_model_dict", {})]

    def _assert_outputs_are_defined(self):
        if not self.__dict__.get("_ml_ready", False):
            return
        bb = set(chain.from_iterable(m.output for m in self.config.ml_model_sources))
        for out in self.outputs:
            if out.alg is None and out.name not in bb:
                raise ValueError(
                    f"Output '{out.name}' was not initialized with an equation, nor is it specified "
                    f"by the provided blackbox models.")
