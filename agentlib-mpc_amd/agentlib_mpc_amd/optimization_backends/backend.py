"""Backend base classes mirroring the reference plugin interface.

Restates `agentlib_mpc/optimization_backends/backend.py`: ``BackendConfig``
(:26-79, results-file validation), ``OptimizationBackend`` (:82-217:
``__init__(config)``, ``register_logger``, ``setup_optimization(var_ref)``,
``solve(now, current_vars) -> Results``, ``update_discretization_options``,
``model_from_config``, ``get_lags_per_variable``) and ``ADMMBackend``
(:223-231, ``coupling_grid``).

When the real ``agentlib_mpc`` package is importable the classes here
subclass the reference ABCs, so ``create_optimization_backend``'s
``isinstance(backend, OptimizationBackend)`` check (`modules/mpc/mpc.py:142`)
holds and the backend drops into an existing agent configuration.
"""

from __future__ import annotations

import abc
import importlib.util
import logging
import os
import pathlib
import sys
from typing import Dict, Optional, Union

import pydantic
from pydantic import ConfigDict

from agentlib_mpc_amd.data_structures import mpc_datamodels
from agentlib_mpc_amd.data_structures.mpc_datamodels import DiscretizationOptions

logger = logging.getLogger(__name__)

try:  # optional: register as a subclass of the reference ABCs when available
    from agentlib_mpc.optimization_backends.backend import (  # type: ignore
        ADMMBackend as _RefADMMBackend,
        OptimizationBackend as _RefOptimizationBackend,
    )
except Exception:  # pragma: no cover - the reference is not installed here
    _RefOptimizationBackend = abc.ABC
    _RefADMMBackend = None


class ConfigurationError(Exception):
    """Raised for invalid backend configurations (agentlib ``ConfigurationError``)."""


class BackendConfig(pydantic.BaseModel):
    model: dict
    discretization_options: DiscretizationOptions
    name: Optional[str] = None
    results_file: Optional[pathlib.Path] = pydantic.Field(default=None)
    save_results: Optional[bool] = pydantic.Field(validate_default=True, default=None)
    overwrite_result_file: Optional[bool] = pydantic.Field(default=False, validate_default=True)
    model_config = ConfigDict(extra="forbid")

    @pydantic.field_validator("results_file")
    @classmethod
    def check_csv(cls, file):
        if file is not None and file.suffix != ".csv":
            raise ConfigurationError(f"Results filename has to be a 'csv' file. Got {file} instead.")
        return file

    @pydantic.field_validator("save_results")
    @classmethod
    def disable_results_if_no_file(cls, save_results, info):
        if save_results is None:
            return bool(info.data.get("results_file"))
        if save_results and info.data.get("results_file") is None:
            raise ConfigurationError("'save_results' was true, however there was no results file provided.")
        return save_results

    @pydantic.field_validator("overwrite_result_file")
    @classmethod
    def check_overwrite(cls, overwrite, info):
        res_file = info.data.get("results_file")
        if res_file and info.data.get("save_results"):
            if overwrite:
                for f in (res_file, mpc_datamodels.stats_path(res_file)):
                    try:
                        os.remove(f)
                    except FileNotFoundError:
                        pass
            elif os.path.isfile(res_file):
                raise FileExistsError(
                    f"Results file {res_file} already exists and will not be overwritten "
                    "automatically. Set 'overwrite_result_file' to True to enable automatic "
                    "overwrite it.")
        return overwrite


def custom_injection(config):
    """Resolve ``{"file": ..., "class_name": ...}`` / class / dotted path to a class
    (agentlib ``custom_injection`` semantics).

    Model files import the reference's model API.  Without the reference installed those
    imports are aliased globally to this package; with it installed, the file is executed
    privately with an import map that resolves them here (:mod:`agentlib_mpc_amd.compat`)."""
    if isinstance(config, type):
        return config
    if isinstance(config, str):
        mod, _, cls = config.rpartition(".")
        return getattr(importlib.import_module(mod), cls)
    if isinstance(config, dict):
        from agentlib_mpc_amd import compat

        if not compat.install_reference_aliases():
            # the reference is installed: its model API must not be what the file binds
            return getattr(compat.load_model_file(config["file"]), config["class_name"])
        file = pathlib.Path(config["file"]).resolve()
        name = f"_mpcx_injected_{abs(hash(str(file)))}"
        if name in sys.modules:
            module = sys.modules[name]
        else:
            spec = importlib.util.spec_from_file_location(name, file)
            module = importlib.util.module_from_spec(spec)
            sys.modules[name] = module
            spec.loader.exec_module(module)
        return getattr(module, config["class_name"])
    raise TypeError(f"Cannot inject a class from {config!r}")


class OptimizationBackend(_RefOptimizationBackend if _RefOptimizationBackend is not abc.ABC else abc.ABC):
    """Base class of optimization backends (`backend.py:82-217`)."""

    _supported_models: dict = {}
    mpc_backend_parameters = ("time_step", "prediction_horizon")
    config_type = BackendConfig

    def __init__(self, config: dict):
        self.logger = logger
        self.config = self.config_type(**config)
        self.model = self.model_from_config(self.config.model)
        self.var_ref = None
        self.stats = {}
        self._created_file = False

    def register_logger(self, logger_: logging.Logger):
        self.logger = logger_

    @abc.abstractmethod
    def setup_optimization(self, var_ref):
        self.var_ref = var_ref

    @abc.abstractmethod
    def solve(self, now, current_vars):
        raise NotImplementedError

    def update_discretization_options(self, opts: dict):
        self.config.discretization_options = self.config.discretization_options.model_copy(update=opts)
        self.setup_optimization(var_ref=self.var_ref)

    def model_from_config(self, model: dict):
        model = dict(model)
        _type = model.pop("type")
        cls = custom_injection(_type)
        from agentlib_mpc_amd import compat

        if compat.is_reference_model_class(cls):
            # a class of the installed reference (given as a class, a dotted path or loaded
            # elsewhere): read it again against this package's model API so it traces
            cls = compat.retrace_model_class(cls)
        instance = cls(**model)
        # `backend.py:94-100`: the reference checks the model against _supported_models
        if self._supported_models and not any(isinstance(instance, m) for m in self._supported_models.values()):
            raise TypeError(
                f"Given model is of type {type(instance)} but should be instance of one of:"
                f"{', '.join(self._supported_models)}")
        return instance

    def get_lags_per_variable(self) -> Dict[str, float]:
        return {}

    def results_file_exists(self) -> bool:
        return self.config.results_file.is_file()

    def results_folder_exists(self) -> bool:
        if self._created_file:
            return True
        if self.results_file_exists():
            self._created_file = True
            return True
        self.config.results_file.parent.mkdir(parents=True, exist_ok=True)
        self._created_file = True
        return False


class ADMMBackend(OptimizationBackend):
    """`backend.py:223-231`."""

    @property
    @abc.abstractmethod
    def coupling_grid(self) -> list:
        raise NotImplementedError


if _RefADMMBackend is not None:  # pragma: no cover - reference not installed here
    _RefADMMBackend.register(ADMMBackend)
