"""Train the two shared networks of the C5 zones (`examples/three_zone_datadriven_admm`)
the way the example does, and write them as serialized ANNs (the reference's
`ml_model.json` format) to ``agentlib_mpc_amd/models/data/ann_t_{air,cca}.json``.

The example trains both ANNs on the fly with keras (`admm_3zone_sim.py:57-65` ->
`training_direct.py:626-642`); the trained weights are not part of the reference, so
they are regenerated here by restating that pipeline (build-container only: the
weather file is read from /root/reference; only the trained weights are committed):

* data (`training_direct.py:285-424`, ``Datagenerator``): the white-box ``Train_NN``
  model (`training_direct.py:151-187`, the ODEs of `models/simulation_model.py:142-165`)
  is simulated for 4 runs x 1000 steps of dt = 1800 s.  Start states 0.9 v + 0.2 v U(0,1)
  with v = 290.15 K (`:358-360`), supply temperatures T_v, T_ahu = 275 + 40 U(0,1),
  d = 400 U(0,1), T_amb / Q_rad from `TRY2015_Aachen_Jahr.dat` (rows of the run's
  segment, `read_weather` :18-36 -- the first data row is skipped and the first 23 rows
  dropped, as there), every other input at its model value (mDot 0.1, mDot_ahu 0.025).
  Inputs are held constant over a step; the step is integrated with RK4 (180 substeps
  of 10 s; the fastest mode has a 525 s time constant) in place of CasADi's cvodes.
* features (`ml_model_trainer.py:498-555`): each input lagged by ``shift(k)`` for
  k < lag, the output column ``T(t+1) - T(t)`` (difference output), rows with a NaN
  dropped, columns in ``column_order`` (lags of `training_direct.py:575-620`); the runs
  are concatenated on one time index as the example does.
* split (`:557-589`): one random permutation, 60 / 20 / 20 % train / validation / test.
* network and fit (`:617-642`): BatchNormalization (keras defaults: eps 1e-3, momentum
  0.99) -> Dense(32, sigmoid) -> Dense(1, linear), MSE, Adam (lr 1e-3), batch 64,
  400 epochs, early stopping with restore_best_weights (patience 500 > epochs, so the
  weights of the best validation epoch are kept), restated in torch fp64.

Run from the repository root: ``python scripts/train_c5_anns.py``.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "agentlib-mpc_amd")]

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
import torch  # noqa: E402

from agentlib_mpc_amd.data_structures.ml_model_datatypes import (  # noqa: E402
    Feature, OutputFeature, column_order, name_with_lag)
from agentlib_mpc_amd.models import examples as ex  # noqa: E402
from agentlib_mpc_amd.models.serialized_ml_model import SerializedANN  # noqa: E402

WEATHER = "/root/reference/examples/three_zone_datadriven_admm/TRY2015_Aachen_Jahr.dat"
OUT_DIR = os.path.join(ROOT, "agentlib-mpc_amd", "agentlib_mpc_amd", "models", "data")
DT = 1800.0
SEED = 20261015 + 5

# Train_NN (`training_direct.py:42-148`): states, inputs and parameters in config order
STATES = ("T_wall", "T_air", "T_CCA_0")
INPUTS = {"T_v": 295.0, "T_ahu": 295.0, "mDot": 0.1, "mDot_ahu": 0.025, "d": 400.0, "T_amb": 290.0,
          "Q_rad": 300.0, "T_set": 298.55, "T_upper": 302.15, "T_lower": 288.15}
PAR = {"cp": 4200.0, "c_BKA": 500000.0, "cw": 518000.0, "cl": 1000.0, "hw": 0.17, "hBKA": 2.0,
       "hFenster": 1.23, "Aw": 13.85, "ABKA": 39.5, "AFenster": 6.6, "mRoom": 60.0}


def read_weather(path):
    """`training_direct.py:18-36` (header at line 33, first data row skipped, iloc[23:])."""
    with open(path) as f:
        contents = [x.strip() for x in f.readlines()][32:]
    title = contents[0].split()
    rows = [r.split() for r in contents[2:]][1:]
    w = pd.DataFrame({t: [float(r[i]) for r in rows] for i, t in enumerate(title)})
    return w.iloc[23:]


def ode(x, u):
    """`training_direct.py:158-179` (= `models/simulation_model.py:144-165`)."""
    T_wall, T_air, T_CCA = x
    p = PAR
    dcca = (p["cp"] * u["mDot"] * (u["T_v"] - T_CCA) / (p["c_BKA"] * p["ABKA"])
            + p["hBKA"] / p["c_BKA"] * (T_air - T_CCA))
    dwall = (p["hw"] / p["cw"] * (T_air - T_wall) + p["hw"] / p["cw"] * (u["T_amb"] - T_wall)
             + u["Q_rad"] / p["cw"])
    m = p["cl"] * p["mRoom"]
    dair = (p["hw"] * p["Aw"] / m * (T_wall - T_air) + p["hBKA"] * p["ABKA"] / m * (T_CCA - T_air)
            + u["d"] / m + (u["T_ahu"] - T_air) * u["mDot_ahu"] / p["mRoom"]
            + p["hFenster"] * p["AFenster"] / m * (u["T_amb"] - T_air) + u["Q_rad"] * p["AFenster"] / m)
    return np.array([dwall, dair, dcca])


def step(x, u, substeps=180):
    h = DT / substeps
    for _ in range(substeps):
        k1 = ode(x, u)
        k2 = ode(x + 0.5 * h * k1, u)
        k3 = ode(x + 0.5 * h * k2, u)
        k4 = ode(x + h * k3, u)
        x = x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
    return x


def generate(rng, weather, n_sim=4, steps=1000):
    """``Datagenerator.generate_data`` (`training_direct.py:346-424`)."""
    amb = weather["t"].to_numpy() + 273.15
    rad = weather["B"].to_numpy()
    runs = []
    for it in range(n_sim):
        true_iter = it % (len(weather) // steps - 1)
        x0 = 0.9 * 290.15 + 0.2 * 290.15 * rng.random(len(STATES))
        rng.random((steps, 1))  # the placeholder column u0 (`:361`), drawn and dropped
        U = {}
        for name, val in INPUTS.items():
            if name == "d":
                U[name] = val * rng.random(steps)
            elif name == "Q_rad":
                U[name] = rad[true_iter * steps:true_iter * steps + steps]
            elif name == "T_amb":
                U[name] = amb[true_iter * steps:true_iter * steps + steps]
            elif name in ("T_v", "T_ahu"):
                U[name] = 275 + 40 * rng.random(steps)
            else:
                U[name] = val * np.ones(steps)
        X = [x0]
        for j in range(steps - 1):
            X.append(step(X[-1], {k: v[j] for k, v in U.items()}))
        X = np.array(X)
        df = pd.DataFrame({s: X[:, i] for i, s in enumerate(STATES)})
        for k, v in U.items():
            df[k] = v
        runs.append(df)
    full = pd.concat(runs)
    full.index = np.arange(0, full.shape[0] * DT, DT)
    return full


def features(data, spec):
    """``create_inputs_and_outputs`` (`ml_model_trainer.py:498-555`)."""
    oname, olag = spec["output"]
    inputs = {n: Feature(name=n, lag=l) for n, l in spec["inputs"].items()}
    outputs = {oname: OutputFeature(name=oname, lag=olag, output_type="difference", recursive=True)}
    lags = dict(spec["inputs"], **{oname: olag})
    X = pd.DataFrame(index=data.index)
    for name, lag in lags.items():
        for k in range(lag):
            X[name_with_lag(name, k)] = data[name].shift(k)
    y = data[oname].shift(-1) - data[oname]
    keep = ~(X.isna().any(axis=1) | y.isna())
    cols = column_order(inputs, outputs)
    return X.loc[keep, cols].to_numpy(), y.loc[keep].to_numpy()[:, None], inputs, outputs, cols


def fit(X, y, rng, epochs=400, batch=64, hidden=32):
    n = X.shape[0]
    perm = rng.permutation(n)
    X, y = X[perm], y[perm]
    n_tr = int(0.6 * n)
    n_va = n_tr + int(0.2 * n)
    torch.manual_seed(SEED)
    net = torch.nn.Sequential(
        torch.nn.BatchNorm1d(X.shape[1], eps=1e-3, momentum=0.01),
        torch.nn.Linear(X.shape[1], hidden), torch.nn.Sigmoid(), torch.nn.Linear(hidden, 1)).double()
    # keras initialisers: glorot-uniform kernels, zero biases
    for lin in (net[1], net[3]):
        torch.nn.init.xavier_uniform_(lin.weight)
        torch.nn.init.zeros_(lin.bias)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3, eps=1e-7)
    Xt, yt = torch.tensor(X[:n_tr]), torch.tensor(y[:n_tr])
    Xv, yv = torch.tensor(X[n_tr:n_va]), torch.tensor(y[n_tr:n_va])
    Xs, ys = torch.tensor(X[n_va:]), torch.tensor(y[n_va:])
    g = torch.Generator().manual_seed(SEED)
    best, best_state = np.inf, None
    for ep in range(epochs):
        net.train()
        order = torch.randperm(n_tr, generator=g)
        for s in range(0, n_tr, batch):
            idx = order[s:s + batch]
            if len(idx) < 2:
                continue
            opt.zero_grad()
            loss = torch.mean((net(Xt[idx]) - yt[idx]) ** 2)
            loss.backward()
            opt.step()
        net.eval()
        with torch.no_grad():
            val = float(torch.mean((net(Xv) - yv) ** 2))
        if val < best:
            best, best_state = val, {k: v.clone() for k, v in net.state_dict().items()}
    net.load_state_dict(best_state)
    net.eval()
    with torch.no_grad():
        test = float(torch.mean((net(Xs) - ys) ** 2))
    return net, {"val_mse": best, "test_mse": test, "n_train": n_tr, "n_validation": n_va - n_tr,
                 "n_test": n - n_va, "epochs": epochs, "batch_size": batch}


def to_serialized(net, inputs, outputs):
    bn, l1, l2 = net[0], net[1], net[3]
    n_in = l1.in_features
    layers = [
        {"class_name": "BatchNormalization", "config": {"axis": -1, "epsilon": 0.001},
         "weights": [bn.weight.detach().numpy(), bn.bias.detach().numpy(),
                     bn.running_mean.numpy(), bn.running_var.numpy()]},
        {"class_name": "Dense", "config": {"units": l1.out_features, "activation": "sigmoid"},
         "weights": [l1.weight.detach().numpy().T.reshape(n_in, -1), l1.bias.detach().numpy()]},
        {"class_name": "Dense", "config": {"units": 1, "activation": "linear"},
         "weights": [l2.weight.detach().numpy().T, l2.bias.detach().numpy()]},
    ]
    return SerializedANN.from_layers(layers, dt=DT, input=inputs, output=outputs)


def main():
    rng = np.random.default_rng(SEED)
    data = generate(rng, read_weather(WEATHER))
    os.makedirs(OUT_DIR, exist_ok=True)
    for fname, spec in (("ann_t_air.json", ex.T_AIR_FEATURES), ("ann_t_cca.json", ex.T_CCA_FEATURES)):
        X, y, inputs, outputs, cols = features(data, spec)
        net, info = fit(X, y, rng)
        ser = to_serialized(net, inputs, outputs)
        ser.training_info = dict(info, columns=cols, script="scripts/train_c5_anns.py", seed=SEED)
        path = os.path.join(OUT_DIR, fname)
        ser.save_serialized_model(path)
        print(path, json.dumps(info))


if __name__ == "__main__":
    main()
