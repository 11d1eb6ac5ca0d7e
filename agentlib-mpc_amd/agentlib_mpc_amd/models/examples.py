"""Models of the benchmark configurations, written against the model API.

Equations restate the reference examples:

* ``OneRoom``      — `examples/one_room_mpc/physical/simple_mpc.py:27-138` (C1, C3)
* ``CooledRoom``   — `examples/4_Room_ADMM_Coordinator/models/room_model.py` (C2)
* ``AirHandler``   — `examples/4_Room_ADMM_Coordinator/models/rlt_model.py` (C2)
* ``ExchangeRoom`` — `examples/exchange_admm/models/room_model.py` (C4)
* ``ExchangeSupply`` — `examples/exchange_admm/models/rlt_model.py` (C4)
"""

from __future__ import annotations

from typing import List

from agentlib_mpc_amd.models.casadi_model import (
    CasadiInput, CasadiModel, CasadiModelConfig, CasadiOutput, CasadiParameter, CasadiState,
)


def _inp(name, value, **kw):
    return CasadiInput(name=name, value=value, **kw)


def _par(name, value, **kw):
    return CasadiParameter(name=name, value=value, **kw)


class OneRoomConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [
        _inp("mDot", 0.0225, unit="m³/s"),      # control: supply air mass flow
        _inp("load", 150, unit="W"),             # disturbance: internal load
        _inp("T_in", 290.15, unit="K"),          # disturbance: supply temperature
        _inp("T_upper", 294.15, unit="K"),       # setting: soft upper bound
    ]
    states: List[CasadiState] = [
        CasadiState(name="T", value=293.15, unit="K"),
        CasadiState(name="T_slack", value=0, unit="K"),  # no ode -> auxiliary
    ]
    parameters: List[CasadiParameter] = [
        _par("cp", 1000), _par("C", 100000), _par("s_T", 1), _par("r_mDot", 1),
    ]
    outputs: List[CasadiOutput] = [CasadiOutput(name="T_out", unit="K")]


class OneRoom(CasadiModel):
    config: OneRoomConfig

    def setup_system(self):
        self.T.ode = self.cp * self.mDot / self.C * (self.T_in - self.T) + self.load / self.C
        self.T_out.alg = self.T
        self.constraints = [(0, self.T + self.T_slack, self.T_upper)]
        ctrl = self.create_sub_objective(expressions=self.mDot, weight=self.r_mDot, name="control_costs")
        slack = self.create_sub_objective(expressions=self.T_slack ** 2, weight=self.s_T, name="temp_slack")
        return self.create_combined_objective(ctrl, slack, normalization=1)


class CooledRoomConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [
        _inp("mDot", 0.0225), _inp("d", 150), _inp("T_in", 290.15),
        _inp("T_set", 294.15), _inp("T_upper", 294.15),
    ]
    states: List[CasadiState] = [CasadiState(name="T", value=293.15)]
    parameters: List[CasadiParameter] = [
        _par("cp", 1000), _par("cZ", 60000), _par("q_T", 1), _par("q_mDot", 1),
    ]


class CooledRoom(CasadiModel):
    config: CooledRoomConfig

    def setup_system(self):
        self.T.ode = self.cp * self.mDot / self.cZ * (self.T_in - self.T) + self.d / self.cZ
        self.constraints = [(0, self.T, self.T_upper)]
        return sum([
            0.0001 * self.q_T * (self.T - self.T_set) ** 2,
            0.0001 * self.q_mDot * (1 / 0.167) ** 2 * self.mDot ** 2,
        ])


ROOMS = 4


class AirHandlerConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [_inp(f"mDot_{i + 1}", 0.0225) for i in range(ROOMS)]
    states: List[CasadiState] = []
    parameters: List[CasadiParameter] = [_par("mDot_max", 0.075)]
    outputs: List[CasadiOutput] = [CasadiOutput(name=f"mDot_out_{i + 1}", value=0.0225) for i in range(ROOMS)]


class AirHandler(CasadiModel):
    config: AirHandlerConfig

    def setup_system(self):
        total = 0
        for i in range(ROOMS):
            self.get(f"mDot_out_{i + 1}").alg = 1 * self.get(f"mDot_{i + 1}")
            total = total + self.get(f"mDot_{i + 1}")
        self.constraints = [(0, total, self.mDot_max)]
        return 0


class ExchangeRoomConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [
        _inp("mDot", 0.0225), _inp("d", 150), _inp("T_in", 290.15),
        _inp("T_set", 294.15), _inp("T_upper", 294.15),
    ]
    states: List[CasadiState] = [CasadiState(name="T", value=293.15)]
    outputs: List[CasadiOutput] = [CasadiOutput(name="mDot_out", value=0.0225)]
    parameters: List[CasadiParameter] = [
        _par("cp", 1000), _par("cZ", 60000), _par("q_T", 1), _par("q_mDot", 1),
    ]


class ExchangeRoom(CasadiModel):
    config: ExchangeRoomConfig

    def setup_system(self):
        self.T.ode = self.cp * self.mDot / self.cZ * (self.T_in - self.T) + self.d / self.cZ
        self.mDot_out.alg = self.mDot
        self.constraints = []
        return sum([
            self.q_T * (self.T - self.T_set) ** 2,
            self.q_mDot * (1 / 0.167) ** 2 * self.mDot ** 2,
        ])


class ExchangeSupplyConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [_inp("mDot", 0.0225, lb=0, ub=0.05)]
    states: List[CasadiState] = []
    parameters: List[CasadiParameter] = [_par("penalty", 1)]
    outputs: List[CasadiOutput] = [CasadiOutput(name="mDot_out", value=0.0225, lb=0, ub=0.05)]


class ExchangeSupply(CasadiModel):
    config: ExchangeSupplyConfig

    def setup_system(self):
        self.mDot_out.alg = -self.mDot
        return self.penalty * self.mDot
