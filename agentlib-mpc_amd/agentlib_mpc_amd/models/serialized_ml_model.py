"""Serialized data-driven models (the ``ml_model_sources`` of a ``CasadiMLModel``).

Restates `agentlib_mpc/models/serialized_ml_model.py`: the pydantic container
``SerializedMLModel`` (:30-153: ``dt``, ``input``, ``output``,
``training_info``, ``model_type``; loading from a dict, JSON string or file)
and ``SerializedANN`` (:155-228: ``structure`` = the keras model JSON,
``weights`` = per-layer lists of arrays).  Keras is not part of this
framework: the ANN structure JSON is read directly (layer ``class_name`` and
``config``), which is all the CasADi translation of the reference uses
(`models/casadi_predictor.py:306-376`).  GPR and linear-regression models are
not on the MI355X path (SURVEY §8a A8/A9 names the ANN only).
"""

from __future__ import annotations

import json
from enum import Enum
from pathlib import Path
from typing import Dict, List, Optional, Union

import numpy as np
from pydantic import BaseModel, ConfigDict, Field

from agentlib_mpc_amd.data_structures.ml_model_datatypes import Feature, OutputFeature


class MLModels(str, Enum):
    ANN = "ANN"
    GPR = "GPR"
    LINREG = "LinReg"
    KerasANN = "KerasANN"


class SerializedMLModel(BaseModel):
    dt: Union[float, int] = Field(title="dt", description="Length of one prediction step in seconds.")
    input: Dict[str, Feature] = Field(default=None, title="input")
    output: Dict[str, OutputFeature] = Field(default=None, title="output")
    training_info: Optional[dict] = Field(default=None, title="Training Info")
    model_type: MLModels
    model_config = ConfigDict(protected_namespaces=(), extra="allow")

    @classmethod
    def load_serialized_model_from_dict(cls, model_data: dict) -> "SerializedMLModel":
        model_type = model_data.get("model_type")
        if model_type in (MLModels.ANN, MLModels.ANN.value):
            return SerializedANN(**model_data)
        raise NotImplementedError(
            f"ML model type {model_type!r} is not supported by the MI355X backend (ANN only).")

    @classmethod
    def load_serialized_model_from_string(cls, json_string: str) -> "SerializedMLModel":
        return cls.load_serialized_model_from_dict(json.loads(json_string))

    @classmethod
    def load_serialized_model_from_file(cls, path: Path) -> "SerializedMLModel":
        with open(path, "r") as f:
            return cls.load_serialized_model_from_dict(json.load(f))

    @classmethod
    def load_serialized_model(cls, model_data: Union[dict, str, Path]) -> "SerializedMLModel":
        if isinstance(model_data, dict):
            return cls.load_serialized_model_from_dict(model_data)
        if isinstance(model_data, (str, Path)) and Path(model_data).exists():
            return cls.load_serialized_model_from_file(Path(model_data))
        return cls.load_serialized_model_from_string(str(model_data))

    def save_serialized_model(self, path: Path):
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        with open(path, "w") as f:
            f.write(self.model_dump_json())


class SerializedANN(SerializedMLModel):
    """Keras-structure JSON + per-layer weight lists (`serialized_ml_model.py:155-228`)."""

    weights: List[list] = Field(default=None, title="weights")
    structure: str = Field(default=None, title="structure")
    model_type: MLModels = MLModels.ANN

    def layer_specs(self) -> List[dict]:
        """Layers with their weights as numpy arrays: ``[{"class_name", "config", "weights"}]``.

        ``InputLayer`` entries of the structure carry no weights and are skipped,
        matching keras' ``model.layers`` (which the weights list was taken from).
        """
        struct = json.loads(self.structure)
        cfg = struct.get("config", {})
        layers = cfg.get("layers", cfg if isinstance(cfg, list) else [])
        layers = [l for l in layers if l.get("class_name") != "InputLayer"]
        if len(layers) != len(self.weights):
            raise ValueError(f"ANN structure has {len(layers)} layers but {len(self.weights)} weight lists")
        return [{"class_name": l["class_name"], "config": l.get("config", {}),
                 "weights": [np.asarray(w, dtype=float) for w in ws]}
                for l, ws in zip(layers, self.weights)]

    @classmethod
    def from_layers(cls, layers: List[dict], dt, input: Dict[str, Feature],
                    output: Dict[str, OutputFeature], training_info: Optional[dict] = None
                    ) -> "SerializedANN":
        """Build from ``[{"class_name", "config", "weights": [arrays]}]`` (keras-equivalent
        structure JSON), e.g. for synthetic networks."""
        structure = json.dumps({"class_name": "Sequential", "config": {
            "name": "sequential", "layers": [{"class_name": l["class_name"], "config": l.get("config", {})}
                                             for l in layers]}})
        weights = [[np.asarray(w, dtype=float).tolist() for w in l["weights"]] for l in layers]
        return cls(structure=structure, weights=weights, dt=dt, input=input, output=output,
                   training_info=training_info)
