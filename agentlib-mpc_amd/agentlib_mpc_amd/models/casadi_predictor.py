"""Symbolic forward pass of serialized ANNs (the NARX models of the ML backends).

Restates the ANN part of `agentlib_mpc/models/casadi_predictor.py`:
activations (``Layer.get_activation`` :255-299), ``Dense`` (:306-336:
``act(x @ W + b)``), ``BatchNormalization`` (:349-376:
``(x - mean) / sqrt(var + eps) * gamma + beta``), ``Normalization``
(:379-398), ``Flatten`` (:339-346) and the sequential ``CasadiANN.predict``.
The input is a row of scalar expressions of the symbolic tracer
(`agentlib_mpc_amd.symbolic`), so the network becomes part of the stage
function that the code generator differentiates and emits as straight-line
HIP; ``predict_numpy`` is the numeric twin used by tests and synthetic-weight
generation.
"""

from __future__ import annotations

import math
from typing import Callable, List, Sequence

import numpy as np

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.models.serialized_ml_model import SerializedANN, SerializedMLModel


def _sigmoid(x):
    return sx.div(sx.ONE, sx.add(sx.ONE, sx.exp(sx.neg(x))))


_SYM_ACT = {
    "sigmoid": _sigmoid,
    "tanh": sx.tanh,
    "relu": lambda x: sx.fmax(sx.ZERO, x),
    "exponential": sx.exp,
    "softplus": lambda x: sx.log(sx.add(sx.ONE, sx.exp(x))),
    "gaussian": lambda x: sx.exp(sx.neg(sx.power(x, 2))),
    "linear": lambda x: x,
}

_NP_ACT = {
    "sigmoid": lambda x: 1.0 / (1.0 + np.exp(-x)),
    "tanh": np.tanh,
    "relu": lambda x: np.maximum(0.0, x),
    "exponential": np.exp,
    "softplus": lambda x: np.log(1.0 + np.exp(x)),
    "gaussian": lambda x: np.exp(-(x ** 2)),
    "linear": lambda x: x,
}


def _activation_name(act) -> str:
    if act is None:
        return "linear"
    if isinstance(act, str):
        if act not in _SYM_ACT:
            raise ValueError(f"Unknown activation function:{act}")
        return act
    # keras 3 serialises activations as {"class_name": ..., "config": ...} dicts
    if isinstance(act, dict) and act.get("class_name") in _SYM_ACT:
        return act["class_name"]
    raise NotImplementedError(f"activation {act!r} is not supported by the MI355X backend")


class CasadiANN:
    """Sequential ANN from a :class:`SerializedANN` (``CasadiANN`` of the reference)."""

    def __init__(self, serialized_model: SerializedANN):
        self.serialized_model = serialized_model
        self.layers = serialized_model.layer_specs()
        self.n_in = None
        self.n_out = None
        for spec in self.layers:
            if spec["class_name"] == "Dense":
                if self.n_in is None:
                    self.n_in = spec["weights"][0].shape[0]
                self.n_out = spec["weights"][0].shape[1]
            elif spec["class_name"] not in ("BatchNormalization", "Normalization", "Flatten", "Dropout"):
                raise NotImplementedError(f"layer {spec['class_name']} is not supported by the MI355X backend")

    # -- symbolic ----------------------------------------------------------------
    def predict(self, inputs: Sequence) -> List[sx.Expr]:
        """Outputs as expressions of ``inputs``.  A normalisation + one smooth hidden
        layer + linear output network (the reference trainer's topology) becomes one
        opaque network node per output (:func:`symbolic.ann_call`, normalisation
        folded into the first layer); anything else is expanded layer by layer."""
        x = [sx.as_expr(v) for v in inputs]
        nets = self._networks()
        if nets is not None:
            return [sx.ann_call(nid, x) for nid in nets]
        for spec in self.layers:
            x = self._layer_sym(spec, x)
        return x

    def _networks(self):
        specs = [s for s in self.layers if s["class_name"] not in ("Flatten", "Dropout")]
        scale = np.ones(self.n_in)
        shift = np.zeros(self.n_in)
        while specs and specs[0]["class_name"] in ("BatchNormalization", "Normalization"):
            spec = specs.pop(0)
            if spec["class_name"] == "BatchNormalization":
                gamma, beta, mean, var = _bn_weights(spec)
                s_ = gamma / np.sqrt(var + float(spec["config"].get("epsilon", 1e-3)))
                t_ = beta - mean * s_
            else:
                mean, var = spec["weights"][0].reshape(-1), spec["weights"][1].reshape(-1)
                s_, t_ = 1.0 / np.sqrt(var), -mean / np.sqrt(var)
            scale, shift = scale * s_, shift * s_ + t_
        if len(specs) != 2 or any(s["class_name"] != "Dense" for s in specs):
            return None
        act1 = _activation_name(specs[0]["config"].get("activation", "linear"))
        act2 = _activation_name(specs[1]["config"].get("activation", "linear"))
        if act1 not in sx._ACTS or act2 != "linear":
            return None
        W1, b1 = specs[0]["weights"][0], _bias(specs[0])
        W2, b2 = specs[1]["weights"][0], _bias(specs[1])
        W1f = scale[:, None] * W1
        b1f = b1 + shift @ W1
        return [sx.register_network(sx.Network(W1f, b1f, W2[:, o], b2[o], act1)) for o in range(W2.shape[1])]

    @staticmethod
    def _layer_sym(spec, x):
        cls, cfg, w = spec["class_name"], spec["config"], spec["weights"]
        if cls == "Dense":
            W = w[0]
            b = w[1] if len(w) >= 2 else np.zeros(W.shape[1])
            act = _SYM_ACT[_activation_name(cfg.get("activation", "linear"))]
            out = []
            for j in range(W.shape[1]):
                acc = sx.const(float(b[j]))
                for i in range(W.shape[0]):
                    if W[i, j] != 0.0:
                        acc = sx.add(acc, sx.mul(float(W[i, j]), x[i]))
                out.append(act(acc))
            return out
        if cls == "BatchNormalization":
            gamma, beta, mean, var = _bn_weights(spec)
            eps = float(cfg.get("epsilon", 1e-3))
            return [sx.add(sx.mul(sx.div(sx.sub(xi, float(m)), math.sqrt(float(v) + eps)), float(g)), float(bt))
                    for xi, g, bt, m, v in zip(x, gamma, beta, mean, var)]
        if cls == "Normalization":
            mean, var = w[0].reshape(-1), w[1].reshape(-1)
            return [sx.div(sx.sub(xi, float(m)), math.sqrt(float(v))) for xi, m, v in zip(x, mean, var)]
        return x  # Flatten / Dropout: identity on one row

    # -- numeric -----------------------------------------------------------------
    def predict_numpy(self, inputs: np.ndarray) -> np.ndarray:
        """Forward pass on rows ``[n, n_in]`` (or one row)."""
        x = np.atleast_2d(np.asarray(inputs, dtype=float))
        for spec in self.layers:
            cls, cfg, w = spec["class_name"], spec["config"], spec["weights"]
            if cls == "Dense":
                b = w[1] if len(w) >= 2 else np.zeros(w[0].shape[1])
                x = _NP_ACT[_activation_name(cfg.get("activation", "linear"))](x @ w[0] + b)
            elif cls == "BatchNormalization":
                gamma, beta, mean, var = _bn_weights(spec)
                x = (x - mean) / np.sqrt(var + float(cfg.get("epsilon", 1e-3))) * gamma + beta
            elif cls == "Normalization":
                x = (x - w[0].reshape(-1)) / np.sqrt(w[1].reshape(-1))
        return x


def _bias(spec):
    w = spec["weights"]
    return w[1] if len(w) >= 2 else np.zeros(w[0].shape[1])


def _bn_weights(spec):
    """gamma, beta, moving mean, moving variance (keras order; scale/center optional)."""
    cfg, w = spec["config"], list(spec["weights"])
    n = w[-1].shape[-1]
    gamma = w.pop(0) if cfg.get("scale", True) else np.ones(n)
    beta = w.pop(0) if cfg.get("center", True) else np.zeros(n)
    mean, var = w[0], w[1]
    return (np.asarray(gamma).reshape(-1), np.asarray(beta).reshape(-1),
            np.asarray(mean).reshape(-1), np.asarray(var).reshape(-1))


class CasadiPredictor:
    """Factory by model type (`casadi_predictor.py` ``CasadiPredictor.from_serialized_model``)."""

    @staticmethod
    def from_serialized_model(serialized_model: SerializedMLModel) -> CasadiANN:
        if isinstance(serialized_model, SerializedANN):
            return CasadiANN(serialized_model)
        raise NotImplementedError(f"{type(serialized_model).__name__} is not supported (ANN only)")
