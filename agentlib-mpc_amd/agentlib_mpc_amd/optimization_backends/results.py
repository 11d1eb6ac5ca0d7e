"""Solve results in the reference's layout.

Restates ``Results`` of `optimization_backends/casadi_/core/discretization.py:31-101`
(matrix over the full time grid, MultiIndex columns ``(parameter|variable|
upper|lower, name)``, ``results[name]`` on the variable's own grid for t >= 0,
``df``, CSV header/stats-line helpers) and the layout builder
``_create_result_format`` (:398-484).
"""

from __future__ import annotations

import dataclasses
from pathlib import Path
from typing import Dict, List

import numpy as np
import pandas as pd


@dataclasses.dataclass
class Results:
    matrix: np.ndarray
    grid: List[float]
    columns: pd.MultiIndex
    stats: dict
    variable_grid_indices: Dict[str, List[int]]
    _variable_name_to_index: Dict[str, int] = None
    objective_values: dict = dataclasses.field(default_factory=dict)

    def __post_init__(self):
        self._variable_name_to_index = self.variable_lookup()

    def __getitem__(self, item: str) -> np.ndarray:
        rows = self.variable_grid_indices[item]
        col = self._variable_name_to_index[item]
        return np.asarray(self.matrix[rows, col]).reshape(-1, 1)

    def variable_lookup(self) -> Dict[str, int]:
        return {label[1]: i for i, label in enumerate(self.columns) if label[0] == "variable"}

    @property
    def df(self) -> pd.DataFrame:
        return pd.DataFrame(self.matrix, index=self.grid, columns=self.columns)

    def write_columns(self, file: Path):
        pd.DataFrame(columns=self.columns).to_csv(file)

    def write_combined_stats_columns(self, file: Path, objective_names: List[str]):
        names = [f"obj_{n}" for n in objective_names] + [f"stats_{n}" for n in self.stats]
        with open(file, "w") as f:
            f.write("," + ",".join(names) + "\n")

    def combined_stats_line(self, index: str, objective_values: dict, objective_names: List[str]) -> str:
        vals = [str(objective_values.get(n, "")) for n in objective_names] + [str(v) for v in self.stats.values()]
        return f'"{index}",' + ",".join(vals) + "\n"

    def write_stats_columns(self, file: Path):
        with open(file, "w") as f:
            f.write("," + ",".join(self.stats) + "\n")

    def stats_line(self, index: str) -> str:
        return f'"{index}",' + ",".join(map(str, self.stats.values())) + "\n"


@dataclasses.dataclass
class ResultLayout:
    """Static part of the result format, computed once per problem structure."""

    full_grid: List[float]
    columns: pd.MultiIndex
    variable_grid_indices: Dict[str, List[int]]
    #: per column block: (kind, group, dim, rows-in-full-grid, grid-columns)
    blocks: list
