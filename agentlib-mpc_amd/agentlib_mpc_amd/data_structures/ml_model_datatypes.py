"""Feature descriptions of data-driven (NARX) models.

Restates `agentlib_mpc/data_structures/ml_model_datatypes.py`: ``OutputType``
(:14-16), ``Feature`` / ``OutputFeature`` (:19-52, including the validator that
forbids non-recursive ``difference`` outputs), ``column_order`` (:118-132, the
order in which lagged features are stacked into the model input) and
``name_with_lag`` (:135-138).  Training-data containers and keras callbacks
belong to the trainer modules, which are out of scope for this backend.
"""

from __future__ import annotations

from enum import Enum
from typing import Dict, List

import pydantic
from pydantic import BaseModel


class OutputType(str, Enum):
    absolute = "absolute"
    difference = "difference"


class Feature(BaseModel):
    name: str
    lag: int = 1


class OutputFeature(Feature):
    output_type: OutputType = pydantic.Field(
        description="'absolute': a forward pass yields the value at the next time step; "
        "'difference': it yields the change, which is added to the current value.")
    recursive: bool = pydantic.Field(
        default=True,
        description="Recursive outputs are also model inputs (state-like); non-recursive "
        "ones model algebraic relationships.")

    @pydantic.field_validator("recursive")
    @classmethod
    def non_recursive_features_have_to_be_absolute(cls, recursive, info):
        if not recursive and info.data.get("output_type") == OutputType.difference:
            raise ValueError(
                f"Output Feature {info.data.get('name')} was specified as a non-recursive feature"
                " for which the difference in output should be learned. This combination is not"
                " allowed. Please set 'output_type' to 'absolute' for non-recursive features.")
        return recursive


def column_order(inputs: Dict[str, Feature], outputs: Dict[str, OutputFeature]) -> List[str]:
    """Order of the (lagged) columns of the model input (`ml_model_datatypes.py:118-132`)."""
    ordered: List[str] = []
    for name, feat in inputs.items():
        for i in range(feat.lag):
            ordered.append(name_with_lag(name, i))
    for name, feat in outputs.items():
        if not feat.recursive:
            continue
        for i in range(feat.lag):
            ordered.append(name_with_lag(name, i))
    return ordered


def name_with_lag(name: str, lag: int) -> str:
    if lag == 0:
        return name
    return f"{name}_{lag}"
