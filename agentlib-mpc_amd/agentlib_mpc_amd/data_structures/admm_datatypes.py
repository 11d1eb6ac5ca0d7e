"""ADMM naming conventions and the per-alias consensus/exchange arithmetic.

Restates `agentlib_mpc/data_structures/admm_datatypes.py`: the prefixes
(:16-23), ``CouplingEntry``/``ExchangeEntry`` (:26-77), the ADMM
``VariableReference`` (:80-109) and the host-side semantics of
``ConsensusVariable`` (:217-282) and ``ExchangeVariable`` (:285-331).  These
host classes are the single-alias reference semantics (and the fleet
driver's bookkeeping); the batched arithmetic runs in the ADMM HIP kernels
(`csrc/admm_kernels.hip`).  Pinned by `tests/golden/admm_golden.json`.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, Hashable, Iterable, List, Optional, Tuple

import numpy as np

from agentlib_mpc_amd.data_structures import mpc_datamodels

ADMM_PREFIX = "admm"
MULTIPLIER_PREFIX = ADMM_PREFIX + "_lambda"
LOCAL_PREFIX = ADMM_PREFIX + "_coupling"
MEAN_PREFIX = ADMM_PREFIX + "_coupling_mean"
LAG_PREFIX = ADMM_PREFIX + "_lag"
EXCHANGE_MULTIPLIER_PREFIX = ADMM_PREFIX + "_exchange_lambda"
EXCHANGE_LOCAL_PREFIX = ADMM_PREFIX + "_exchange"
EXCHANGE_MEAN_PREFIX = ADMM_PREFIX + "_exchange_mean"
PENALTY_FACTOR = "penalty_factor"


@dataclasses.dataclass
class CouplingEntry:
    name: str

    @property
    def local(self):
        return f"{LOCAL_PREFIX}_{self.name}"

    @property
    def mean(self):
        return f"{MEAN_PREFIX}_{self.name}"

    @property
    def multiplier(self):
        return f"{MULTIPLIER_PREFIX}_{self.name}"

    @property
    def lagged(self):
        return f"{LAG_PREFIX}_{self.name}"

    def admm_variables(self):
        return [self.local, self.mean, self.multiplier, self.lagged]


@dataclasses.dataclass
class ExchangeEntry:
    name: str

    @property
    def local(self):
        return f"{EXCHANGE_LOCAL_PREFIX}_{self.name}"

    @property
    def mean_diff(self):
        return f"{EXCHANGE_MEAN_PREFIX}_{self.name}"

    @property
    def multiplier(self):
        return f"{EXCHANGE_MULTIPLIER_PREFIX}_{self.name}"

    @property
    def lagged(self):
        return f"{LAG_PREFIX}_{self.name}"

    def admm_variables(self):
        return [self.local, self.mean_diff, self.multiplier, self.lagged]


@dataclasses.dataclass
class VariableReference(mpc_datamodels.VariableReference):
    couplings: List[CouplingEntry] = dataclasses.field(default_factory=list)
    exchange: List[ExchangeEntry] = dataclasses.field(default_factory=list)

    def all_variables(self) -> List[str]:
        d = dict(self.__dict__)
        coup = d.pop("couplings")
        exch = d.pop("exchange")
        base = [v for vals in d.values() for v in vals]
        return base + [c.name for c in coup + exch]


def coupling_alias(alias: str) -> str:
    return f"{LOCAL_PREFIX}_{alias}"


def exchange_alias(alias: str) -> str:
    return f"{EXCHANGE_LOCAL_PREFIX}_{alias}"


Source = Hashable


@dataclasses.dataclass
class CouplingVariable:
    """Per-alias state kept by the coordinator (`admm_datatypes.py:161-214`)."""

    local_trajectories: Dict[Source, list] = dataclasses.field(default_factory=dict)
    mean_trajectory: list = dataclasses.field(default_factory=lambda: [0])
    delta_mean: np.ndarray = dataclasses.field(default_factory=lambda: np.array([0]))
    primal_residual: np.ndarray = dataclasses.field(default_factory=lambda: np.array([0]))

    def _relevant_sources(self, sources: Optional[Iterable[Source]]) -> list:
        if sources is None:
            return list(self.local_trajectories)
        wanted = set(sources)
        return [s for s in self.local_trajectories if s in wanted]

    @property
    def participants(self):
        return list(self.local_trajectories)

    def flat_locals(self, sources=None) -> list:
        return [self.local_trajectories[s] for s in self._relevant_sources(sources)]

    def get_residual(self, rho: float) -> Tuple[np.ndarray, np.ndarray]:
        return np.asarray(self.primal_residual).flatten(), (rho * np.asarray(self.delta_mean)).flatten()


@dataclasses.dataclass
class ConsensusVariable(CouplingVariable):
    multipliers: Dict[Source, list] = dataclasses.field(default_factory=dict)

    def update_mean_trajectory(self, sources=None):
        src = self._relevant_sources(sources)
        if not src:
            return
        mean = np.mean(np.array([self.local_trajectories[s] for s in src]), axis=0)
        self.delta_mean = self.mean_trajectory - mean
        self.mean_trajectory = list(mean)

    def update_multipliers(self, rho: float, sources=None):
        src = self._relevant_sources(sources)
        if not src:
            return
        traj = np.array([self.local_trajectories[s] for s in src])
        lam = np.array([self.multipliers[s] for s in src])
        self.primal_residual = np.array(self.mean_trajectory) - traj
        new = lam - rho * self.primal_residual
        for i, s in enumerate(src):
            self.multipliers[s] = new[i, :].tolist()

    def flat_multipliers(self, sources=None) -> list:
        return [self.multipliers[s] for s in self._relevant_sources(sources)]

    def shift_values_by_one(self, horizon: int):
        m = self.mean_trajectory
        k = int(len(m) / horizon)
        self.mean_trajectory = m[k:] + m[-k:]
        for key, mul in self.multipliers.items():
            self.multipliers[key] = mul[k:] + mul[-k:]


@dataclasses.dataclass
class ExchangeVariable(CouplingVariable):
    diff_trajectories: Dict[Source, list] = dataclasses.field(default_factory=dict)
    multiplier: list = dataclasses.field(default_factory=list)

    def update_diff_trajectories(self, sources=None):
        src = self._relevant_sources(sources)
        if not src:
            return
        mean = np.mean(np.array([self.local_trajectories[s] for s in src]), axis=0)
        self.delta_mean = self.mean_trajectory - mean
        self.mean_trajectory = list(mean)
        for s in src:
            self.diff_trajectories[s] = list(self.local_trajectories[s] - mean)

    def update_multiplier(self, rho: float):
        self.primal_residual = np.array(self.mean_trajectory)
        self.multiplier = list(self.multiplier + rho * self.primal_residual)

    def shift_values_by_one(self, horizon: int):
        k = int(len(self.multiplier) / horizon)
        self.multiplier = self.multiplier[k:] + self.multiplier[-k:]
        for key, diff in self.diff_trajectories.items():
            self.diff_trajectories[key] = diff[k:] + diff[-k:]
