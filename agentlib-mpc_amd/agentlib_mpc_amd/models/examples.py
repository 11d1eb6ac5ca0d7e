"""Models of the benchmark configurations, written against the model API.

Equations restate the reference examples:

* ``OneRoom``      — `examples/one_room_mpc/physical/simple_mpc.py:27-138` (C1, C3)
* ``CooledRoom``   — `examples/4_Room_ADMM_Coordinator/models/room_model.py` (C2)
* ``AirHandler``   — `examples/4_Room_ADMM_Coordinator/models/rlt_model.py` (C2)
* ``ExchangeRoom`` — `examples/exchange_admm/models/room_model.py` (C4)
* ``ExchangeSupply`` — `examples/exchange_admm/models/rlt_model.py` (C4)
* ``RoomCCA``      — `examples/three_zone_datadriven_admm/models/Room_model.py` (C5, NARX)
* ``RNGRoom``      — `examples/Estimators/mhe_example.py:21-170` (moving horizon estimation)
"""

from __future__ import annotations

import os
from typing import List, Optional

import numpy as np

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


class OneRoomDUConfig(OneRoomConfig):
    parameters: List[CasadiParameter] = [
        _par("cp", 1000), _par("C", 100000), _par("s_T", 1), _par("r_mDot", 1), _par("r_delta_mDot", 1),
    ]


class OneRoomDU(CasadiModel):
    """`examples/one_room_mpc/physical/with_change_control_penalty.py:98-133`:
    the one-room model with a change penalty on the supply mass flow."""

    config: OneRoomDUConfig

    def setup_system(self):
        self.T.ode = self.cp * self.mDot / self.C * (self.T_in - self.T) + self.load / self.C
        self.T_out.alg = self.T
        self.constraints = [(0, self.T + self.T_slack, self.T_upper)]
        obj1 = self.create_sub_objective(expressions=self.mDot, weight=self.r_mDot, name="control_costs")
        obj2 = self.create_sub_objective(expressions=self.T_slack ** 2, weight=self.s_T, name="temp_slack")
        obj3 = self.create_change_penalty(expressions=self.mDot, name="delta_control_penalty")
        return self.create_combined_objective(obj1, obj2, obj3 * self.r_delta_mDot, normalization=1)


class SwitchRoomConfig(OneRoomConfig):
    parameters: List[CasadiParameter] = [
        _par("cp", 1000), _par("C", 100000), _par("s_T", 1), _par("r_mDot", 1), _par("r_mDot2", 1),
        _par("switch", 600, unit="s"),
    ]
    outputs: List[CasadiOutput] = [CasadiOutput(name="T_out", unit="K"), CasadiOutput(name="switch_test", unit="-")]


class SwitchRoom(CasadiModel):
    """`examples/one_room_mpc/physical/simple_mpc_time_dependent_obj.py:108-165`:
    the one-room model with a time-dependent (conditional) objective."""

    config: SwitchRoomConfig

    def setup_system(self):
        from agentlib_mpc_amd.models.casadi_model import ca

        self.T.ode = self.cp * self.mDot / self.C * (self.T_in - self.T) + self.load / self.C
        self.T_out.alg = self.T
        self.constraints = [(0, self.T + self.T_slack, self.T_upper)]
        obj1_mDot = self.create_sub_objective(expressions=self.mDot, weight=self.r_mDot, name="mDot_cost_normal")
        obj1_slack = self.create_sub_objective(expressions=self.T_slack ** 2, weight=self.s_T,
                                               name="temperature_slack")
        objective1 = self.create_combined_objective(obj1_mDot, obj1_slack, normalization=10)
        obj2_mDot = self.create_sub_objective(expressions=self.mDot, weight=self.r_mDot2, name="mDot_cost_doubled")
        obj2_slack = self.create_sub_objective(expressions=self.T_slack ** 2, name="temperature_slack_2")
        objective2 = self.create_combined_objective(obj2_mDot) + self.create_combined_objective(obj2_slack) * self.s_T
        condition = self.time < self.switch.sym
        objective = self.create_conditional_objective((condition, objective1), default_objective=objective2)
        self.switch_test.alg = ca.if_else(self.time < self.switch.sym, 1, 2)
        return objective


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


# ---------------------------------------------------------------------------
# C5: three-zone data-driven ADMM (`examples/three_zone_datadriven_admm`)
# ---------------------------------------------------------------------------

from agentlib_mpc_amd.models.casadi_ml_model import CasadiMLModel, CasadiMLModelConfig  # noqa: E402


class RoomCCAConfig(CasadiMLModelConfig):
    """`examples/three_zone_datadriven_admm/models/Room_model.py:13-81`."""

    inputs: List[CasadiInput] = [
        _inp("T_v", 293.15, unit="K"), _inp("T_ahu", 293.15, unit="K"),
        _inp("mDot", 0.1), _inp("mDot_ahu", 0.025),
        _inp("d", 0, unit="W"), _inp("T_amb", 299, unit="K"), _inp("Q_rad", 0, unit="W/m²"),
        _inp("T_set", 298.55, unit="K"), _inp("T_upper", 301.15, unit="K"), _inp("T_lower", 288.15, unit="K"),
    ]
    states: List[CasadiState] = [
        CasadiState(name="T_air", value=290.15, unit="K"),
        CasadiState(name="T_CCA_0", value=293.15, unit="K"),
        CasadiState(name="T_slack", value=0, unit="K"),  # no model -> auxiliary
    ]
    parameters: List[CasadiParameter] = [_par("q_T", 1), _par("s_T", 1)]
    outputs: List[CasadiOutput] = [
        CasadiOutput(name="T_CCA_out", value=293.15, unit="K"),
        CasadiOutput(name="T_air_out", value=293.15, unit="K"),
    ]


class RoomCCA(CasadiMLModel):
    """`Room_model.py:84-105`: T_air and T_CCA_0 are predicted by two ANNs."""

    config: RoomCCAConfig

    def setup_system(self):
        self.T_CCA_out.alg = self.T_CCA_0
        self.T_air_out.alg = self.T_air
        self.constraints = [(self.T_lower, self.T_air + self.T_slack, self.T_upper)]
        return sum([
            1 * 10 * self.q_T * (self.T_air - self.T_set) ** 2,
            1 * 10 * self.s_T * self.T_slack ** 2,
        ])


#: ANN feature lags of `examples/three_zone_datadriven_admm/training_direct.py:575-620`
T_AIR_FEATURES = {"inputs": {"T_CCA_0": 1, "T_ahu": 1, "mDot_ahu": 1, "d": 2, "T_amb": 1, "Q_rad": 2},
                  "output": ("T_air", 1)}
T_CCA_FEATURES = {"inputs": {"T_air": 1, "T_v": 3, "d": 1, "mDot": 2},
                  "output": ("T_CCA_0", 1)}
#: (typical value, spread) of each feature, used for the BatchNormalization statistics
_FEATURE_SCALE = {"T_CCA_0": (295.0, 2.0), "T_ahu": (295.0, 3.0), "mDot_ahu": (0.025, 0.01),
                  "d": (100.0, 60.0), "T_amb": (299.0, 5.0), "Q_rad": (100.0, 80.0),
                  "T_air": (296.0, 2.0), "T_v": (295.0, 4.0), "mDot": (0.1, 0.04)}


def synthetic_ann(features: dict, seed: int, hidden: int = 32, dt: float = 1800.0):
    """A seeded ANN with the reference trainer's topology
    (`ml_model_trainer.py:617-626`: BatchNormalization -> Dense(32, sigmoid) ->
    Dense(1, linear)) on the lagged features of the three-zone example.  The
    trained networks of the example are produced at run time by keras
    (`admm_3zone_sim.py:57-65`) and are not part of the reference, so the C5
    weights are synthetic; the output weights are scaled so one step changes the
    temperature by at most a few tenths of a kelvin."""
    from agentlib_mpc_amd.data_structures.ml_model_datatypes import Feature, OutputFeature, column_order
    from agentlib_mpc_amd.models.serialized_ml_model import SerializedANN

    rng = np.random.default_rng(seed)
    inputs = {n: Feature(name=n, lag=l) for n, l in features["inputs"].items()}
    oname, olag = features["output"]
    outputs = {oname: OutputFeature(name=oname, lag=olag, output_type="difference", recursive=True)}
    cols = column_order(inputs, outputs)
    base = [c.rsplit("_", 1)[0] if c not in _FEATURE_SCALE else c for c in cols]
    mean = np.array([_FEATURE_SCALE[b][0] for b in base])
    var = np.array([_FEATURE_SCALE[b][1] ** 2 for b in base])
    n_in = len(cols)
    W1 = rng.normal(0.0, 1.0 / np.sqrt(n_in), (n_in, hidden))
    b1 = rng.normal(0.0, 0.1, hidden)
    W2 = rng.normal(0.0, 0.6 / np.sqrt(hidden), (hidden, 1))
    b2 = np.array([-0.5 * W2[:, 0].sum()])  # zero-centred output at sigmoid midpoints
    layers = [
        {"class_name": "BatchNormalization", "config": {"axis": -1, "epsilon": 0.001},
         "weights": [np.ones(n_in), np.zeros(n_in), mean, var]},
        {"class_name": "Dense", "config": {"units": hidden, "activation": "sigmoid"}, "weights": [W1, b1]},
        {"class_name": "Dense", "config": {"units": 1, "activation": "linear"}, "weights": [W2, b2]},
    ]
    return SerializedANN.from_layers(layers, dt=dt, input=inputs, output=outputs)


def trained_anns():
    """The two networks of the C5 zones trained as the example trains them
    (`three_zone_datadriven_admm/training_direct.py:553-642`: white-box simulation data,
    BatchNormalization -> Dense(32, sigmoid) -> Dense(1), MSE/Adam, 400 epochs), produced
    by ``scripts/train_c5_anns.py`` and stored in the reference's ``ml_model.json`` format."""
    from agentlib_mpc_amd.models.serialized_ml_model import SerializedMLModel

    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
    return [SerializedMLModel.load_serialized_model_from_file(os.path.join(here, f))
            for f in ("ann_t_air.json", "ann_t_cca.json")]


def room_cca_anns(seed: Optional[int] = None):
    """The two shared networks of the C5 zones (T_air and T_CCA_0): the trained ones by
    default, seeded synthetic ones of the same topology when ``seed`` is given."""
    if seed is None:
        return trained_anns()
    return [synthetic_ann(T_AIR_FEATURES, seed), synthetic_ann(T_CCA_FEATURES, seed + 1)]


class ThreeZoneAHUConfig(CasadiModelConfig):
    """`examples/three_zone_datadriven_admm/models/AHU.py:4-75` (air handling unit of 3 zones)."""

    inputs: List[CasadiInput] = [
        _inp("mDot_0", 0.025), _inp("T_amb", 295, unit="K"),
        _inp("T_ahu1", 294, unit="K"), _inp("T_ahu2", 294, unit="K"), _inp("T_ahu3", 294, unit="K"),
        _inp("T_room1", 299, unit="K"), _inp("T_room2", 299, unit="K"), _inp("T_room3", 299, unit="K"),
    ]
    states: List[CasadiState] = []
    parameters: List[CasadiParameter] = [_par("r_T_v", 1), _par("cl", 1000, unit="J/kg*K")]
    outputs: List[CasadiOutput] = [
        CasadiOutput(name="T_ahu_out1", value=293), CasadiOutput(name="T_ahu_out2", value=293),
        CasadiOutput(name="T_ahu_out3", value=293),
        CasadiOutput(name="W1", value=200), CasadiOutput(name="W2", value=200), CasadiOutput(name="W3", value=200),
    ]


class ThreeZoneAHU(CasadiModel):
    """`AHU.py:78-130`: supply temperatures of three zones, smoothed |power| cost."""

    config: ThreeZoneAHUConfig

    def setup_system(self):
        zones = ((self.T_ahu1, self.T_room1, self.T_ahu_out1, self.W1),
                 (self.T_ahu2, self.T_room2, self.T_ahu_out2, self.W2),
                 (self.T_ahu3, self.T_room3, self.T_ahu_out3, self.W3))
        terms = []
        for t_ahu, t_room, out, w in zones:
            out.alg = 1 * t_ahu
            w.alg = self.cl * self.mDot_0 * (t_ahu - (t_room + self.T_amb) / 2)
            terms.append(0.1 * 0.001 * self.r_T_v
                         * ((self.cl * self.mDot_0 * (t_ahu - (t_room + self.T_amb) / 2)) ** 2 + 0.02) ** 0.5)
        self.constraints = []
        return sum(terms)


class TempControllerConfig(CasadiModelConfig):
    """`examples/three_zone_datadriven_admm/models/CCA.py:4-50` (concrete core activation supply)."""

    inputs: List[CasadiInput] = [
        _inp("mDot_0", 0.1), _inp("T_v", 294, unit="K"),
        _inp("T_r1", 296), _inp("T_r2", 296), _inp("T_r3", 296),
    ]
    states: List[CasadiState] = []
    parameters: List[CasadiParameter] = [_par("r_T_v", 1), _par("cp", 4200, unit="J/kg*K")]
    outputs: List[CasadiOutput] = [
        CasadiOutput(name="T_v_out", value=293), CasadiOutput(name="T_v_out2", value=293),
        CasadiOutput(name="T_v_out3", value=293),
        CasadiOutput(name="W1", value=200), CasadiOutput(name="W2", value=200), CasadiOutput(name="W3", value=200),
    ]


class TempController(CasadiModel):
    """`CCA.py:53-88`: one supply temperature for three zones."""

    config: TempControllerConfig

    def setup_system(self):
        self.T_v_out.alg = 1 * self.T_v
        self.T_v_out2.alg = 1 * self.T_v
        self.T_v_out3.alg = 1 * self.T_v
        self.W1.alg = self.cp * self.mDot_0 * (self.T_v - self.T_r1)
        self.W2.alg = self.cp * self.mDot_0 * (self.T_v - self.T_r2)
        self.W3.alg = self.cp * self.mDot_0 * (self.T_v - self.T_r3)
        self.constraints = []
        return sum(0.1 * 0.001 * self.r_T_v * ((self.cp * self.mDot_0 * (self.T_v - t_r)) ** 2 + 0.02) ** 0.5
                   for t_r in (self.T_r1, self.T_r2, self.T_r3))


class RNGRoomConfig(CasadiModelConfig):
    inputs: List[CasadiInput] = [
        _inp("mDot", 0.22, unit="kg/s"), _inp("load", 150, unit="W"), _inp("T_in", 290.15, unit="K"),
        _inp("T_ambient", 28, unit="K"), _inp("T_upper", 22, unit="K"),
    ]
    states: List[CasadiState] = [
        CasadiState(name="T", value=22, unit="K"),
        CasadiState(name="T_wall", value=23, unit="K"),
        CasadiState(name="T_slack", value=0, unit="K"),  # no ode -> auxiliary
    ]
    parameters: List[CasadiParameter] = [
        _par("cp", 1005), _par("rho", 1.2), _par("full_capacity_from_volume_factor", 5.5),
        _par("C_Wall", 4_569_348), _par("RZone_Wall", 0.0129), _par("R_hull_amb", 0.1128),
        _par("V", 59), _par("s_T", 1), _par("r_mDot", 1),
    ]
    outputs: List[CasadiOutput] = [
        CasadiOutput(name="T_out", unit="K"), CasadiOutput(name="cooling"), CasadiOutput(name="power_wall2zone"),
    ]


class RNGRoom(CasadiModel):
    """`examples/Estimators/mhe_example.py:21-170`: zone + wall model whose
    capacity factor the moving horizon estimator identifies."""

    config: RNGRoomConfig

    def setup_system(self):
        power_wall2zone = (self.T_wall - self.T) / self.RZone_Wall
        air_cooling = self.cp * self.mDot * (self.T_in - self.T)
        C_zone = self.rho * self.cp * self.V * self.full_capacity_from_volume_factor
        self.T.ode = (self.load + air_cooling + power_wall2zone) / C_zone
        power_wall2amb = (self.T_wall - self.T_ambient) / self.R_hull_amb
        self.T_wall.ode = -(power_wall2amb + power_wall2zone) / self.C_Wall
        self.T_out.alg = self.T
        self.cooling.alg = air_cooling
        self.power_wall2zone.alg = power_wall2zone
        self.constraints = [(0, self.T + self.T_slack, self.T_upper)]
        return sum([self.r_mDot * self.mDot, self.s_T * self.T_slack ** 2])


class RNGRoomMHEConfig(RNGRoomConfig):
    states: List[CasadiState] = [
        CasadiState(name="T", value=22, unit="K"),
        CasadiState(name="T_wall", value=23, unit="K"),
        CasadiState(name="T_slack", value=0, unit="K", lb=-50),
    ]


class RNGRoomMHE(RNGRoom):
    """``RNGRoom`` with the soft-constraint slack bounded below.  In the estimator
    the slack has no cost, so with the example's unbounded slack every value below
    ``T_upper - T`` is optimal and the solver returns an arbitrary point of that
    ray; with a finite lower bound the barrier problems have a unique solution
    (the middle of the feasible interval) that two interior-point solvers agree on."""

    config: RNGRoomMHEConfig


class FixtureModelConfig(CasadiModelConfig):
    """The reference test-suite model (`tests/fixtures/casadi_test_model.py:13-34`)."""

    parameters: List[CasadiParameter] = [_par("par", 12, unit="kg"), _par("par2", 10, unit="kg")]
    states: List[CasadiState] = [CasadiState(name="state", value=290, unit="K")]
    inputs: List[CasadiInput] = [_inp("myctrl", 100, unit="W"), _inp("disturbance", 280, unit="K")]
    outputs: List[CasadiOutput] = [CasadiOutput(name="myout", value=100)]


class FixtureModel(CasadiModel):
    """`tests/fixtures/casadi_test_model.py:37-47`: one unstable state driven by a control
    and a disturbance, its value as output, quadratic tracking cost (deprecated plain
    objective return)."""

    config: FixtureModelConfig

    def setup_system(self):
        self.state.ode = self.myctrl + self.par * (self.state - self.disturbance) - self.par2
        self.myout.alg = self.state
        return (self.state - 290) ** 2


class CubicRoomConfig(CasadiModelConfig):
    """A zone temperature with an algebraic quantity on a cubic characteristic: the
    restoration-phase parity case (the cold guess, the middle of the bounds, sits in the
    basin of the characteristic's local infeasibility minimum)."""

    states: List[CasadiState] = [CasadiState(name="T", value=295.0, unit="K"),
                                 CasadiState(name="z", value=0.0, lb=-5.0, ub=2.6)]
    inputs: List[CasadiInput] = [_inp("u", 0.0, unit="K/s")]


class CubicRoom(CasadiModel):
    """``T' = u - 0.01 (T - 290)``, ``z^3 - 3 z - 5 = 0`` at every point, cost ``(T - 290)^2``."""

    config: CubicRoomConfig

    def setup_system(self):
        self.T.ode = self.u - 0.01 * (self.T - 290)
        self.constraints = [(0, self.z ** 3 - 3 * self.z - 5, 0)]
        return (self.T - 290) ** 2
