"""Generate golden vectors by executing the reference's own pure-numpy modules.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_golden.py

The reference package cannot be imported normally (``agentlib``, ``casadi``,
``orjson`` are not installed), so the package roots and the three external
modules these files touch are stubbed.  The modules executed are
`agentlib_mpc/utils/sampling.py` and `agentlib_mpc/data_structures/admm_datatypes.py`
(+ the `interpolation.py`, `coordinator_datatypes.py`, `mpc_datamodels.py` they
import).  Only inputs and outputs are written (JSON); no reference source is copied.
"""

from __future__ import annotations

import importlib.util
import json
import pathlib
import sys
import types

import numpy as np
import pandas as pd

REF = pathlib.Path("/root/reference/agentlib_mpc")
OUT = pathlib.Path(__file__).resolve().parent


def _stub_packages():
    for name in ("agentlib", "agentlib.core", "agentlib.core.module", "agentlib.core.datamodels",
                 "agentlib.core.errors", "orjson"):
        sys.modules.setdefault(name, types.ModuleType(name))
    al = sys.modules["agentlib"]
    al.Source = object
    core = sys.modules["agentlib.core"]

    class AgentVariable:  # attrs-subclassable stand-in
        pass

    core.AgentVariable = AgentVariable
    sys.modules["agentlib.core.module"].BaseModuleConfigClass = object
    sys.modules["agentlib.core.errors"].ConfigurationError = Exception
    sys.modules["orjson"].dumps = json.dumps
    sys.modules["orjson"].loads = json.loads
    sys.modules["orjson"].OPT_SERIALIZE_NUMPY = 0
    sys.modules["orjson"].OPT_SERIALIZE_DATACLASS = 0
    for pkg in ("agentlib_mpc", "agentlib_mpc.data_structures", "agentlib_mpc.utils"):
        m = types.ModuleType(pkg)
        m.__path__ = [str(REF / pkg.split(".", 1)[1].replace(".", "/"))] if "." in pkg else [str(REF)]
        sys.modules[pkg] = m


def _load(modname: str, rel: str):
    spec = importlib.util.spec_from_file_location(modname, REF / rel)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[modname] = mod
    spec.loader.exec_module(mod)
    parent, _, leaf = modname.rpartition(".")
    setattr(sys.modules[parent], leaf, mod)
    return mod


def _clean(x):
    if isinstance(x, (np.floating, float)):
        return float(x)
    if isinstance(x, (list, tuple, np.ndarray)):
        return [_clean(v) for v in x]
    return x


def sampling_cases(sampling, interp):
    rng = np.random.default_rng(20261015)
    cases = []
    grids = [[0, 300, 600, 900], [5, 12, 20, 28, 35], list(np.linspace(0, 4500, 16)),
             [0, 15, 30, 45, 60, 75, 90, 105, 120]]
    for method in ("linear", "previous", "mean_over_interval"):
        for gi, grid in enumerate(grids):
            for current in (0.0, 30.0, 250.0):
                idx = np.sort(rng.choice(np.arange(0, 5000, 10), size=12, replace=False)).astype(float)
                vals = rng.normal(size=12)
                sr = pd.Series(vals, index=idx)
                try:
                    out = sampling.sample(trajectory=sr, grid=grid, current=current,
                                          method=interp.InterpolationMethods(method))
                except Exception as e:  # record the error type as the expected outcome
                    out = {"error": type(e).__name__}
                cases.append({"kind": "series", "index": idx.tolist(), "values": vals.tolist(),
                              "grid": _clean(grid), "current": current, "method": method,
                              "expected": _clean(out)})
    for scalar in (3.5, 0, -1e19):
        cases.append({"kind": "scalar", "value": scalar, "grid": [0, 1, 2], "current": 0.0,
                      "method": "linear", "expected": _clean(sampling.sample(scalar, [0, 1, 2]))})
    cases.append({"kind": "list", "value": [1.0, 2.0, 3.0], "grid": [0, 1, 2], "current": 0.0,
                  "method": "linear", "expected": _clean(sampling.sample([1.0, 2.0, 3.0], [0, 1, 2]))})
    return cases


def admm_cases(adt):
    rng = np.random.default_rng(20261016)
    out = []
    for trial in range(6):
        n_src, T = int(rng.integers(2, 6)), int(rng.integers(3, 12))
        rho = float(rng.uniform(0.1, 100))
        srcs = [f"agent_{i}" for i in range(n_src)]
        cv = adt.ConsensusVariable()
        locals0 = {s: rng.normal(size=T).tolist() for s in srcs}
        cv.local_trajectories = dict(locals0)
        cv.multipliers = {s: rng.normal(size=T).tolist() for s in srcs}
        mult0 = {s: list(v) for s, v in cv.multipliers.items()}
        active = [s for s in srcs if rng.uniform() > 0.25] or srcs[:1]
        cv.update_mean_trajectory(sources=active)
        mean1 = list(cv.mean_trajectory)
        dmean1 = np.asarray(cv.delta_mean).tolist()
        cv.update_multipliers(rho=rho, sources=active)
        prim, dual = cv.get_residual(rho=rho)
        # second round (delta_mean against a real previous mean)
        locals1 = {s: rng.normal(size=T).tolist() for s in srcs}
        cv.local_trajectories = dict(locals1)
        cv.update_mean_trajectory(sources=active)
        mean2 = list(cv.mean_trajectory)
        dmean2 = np.asarray(cv.delta_mean).tolist()
        cv.update_multipliers(rho=rho, sources=active)
        prim2, dual2 = cv.get_residual(rho=rho)
        mult2 = {s: list(v) for s, v in cv.multipliers.items()}
        cv.shift_values_by_one(horizon=T)
        out.append({
            "type": "consensus", "T": T, "rho": rho, "sources": srcs, "active": active,
            "locals0": locals0, "multipliers0": mult0, "locals1": locals1,
            "mean1": _clean(mean1), "delta_mean1": _clean(dmean1),
            "primal1": _clean(prim), "dual1": _clean(dual),
            "mean2": _clean(mean2), "delta_mean2": _clean(dmean2),
            "primal2": _clean(prim2), "dual2": _clean(dual2), "multipliers2": _clean(mult2),
            "shifted_mean": _clean(cv.mean_trajectory),
            "shifted_multipliers": _clean(cv.multipliers),
        })
    for trial in range(4):
        n_src, T = int(rng.integers(2, 8)), int(rng.integers(3, 12))
        rho = float(rng.uniform(0.1, 1e4))
        srcs = [f"agent_{i}" for i in range(n_src)]
        ev = adt.ExchangeVariable()
        locals0 = {s: rng.normal(size=T).tolist() for s in srcs}
        ev.local_trajectories = {s: np.asarray(v) for s, v in locals0.items()}
        ev.multiplier = rng.normal(size=T).tolist()
        mult0 = list(ev.multiplier)
        ev.update_diff_trajectories()
        mean1 = list(ev.mean_trajectory)
        dmean1 = np.asarray(ev.delta_mean).tolist()
        diffs1 = {s: _clean(v) for s, v in ev.diff_trajectories.items()}
        ev.update_multiplier(rho=rho)
        prim, dual = ev.get_residual(rho=rho)
        mult1 = list(ev.multiplier)
        ev.shift_values_by_one(horizon=T)
        out.append({
            "type": "exchange", "T": T, "rho": rho, "sources": srcs, "locals0": locals0,
            "multiplier0": mult0, "mean1": _clean(mean1), "delta_mean1": _clean(dmean1),
            "diffs1": diffs1, "multiplier1": _clean(mult1), "primal1": _clean(prim),
            "dual1": _clean(dual), "shifted_multiplier": _clean(ev.multiplier),
            "shifted_diffs": {s: _clean(v) for s, v in ev.diff_trajectories.items()},
        })
    return out


def main():
    _stub_packages()
    interp = _load("agentlib_mpc.data_structures.interpolation", "data_structures/interpolation.py")
    sampling = _load("agentlib_mpc.utils.sampling", "utils/sampling.py")
    _load("agentlib_mpc.data_structures.coordinator_datatypes", "data_structures/coordinator_datatypes.py")
    _load("agentlib_mpc.data_structures.mpc_datamodels", "data_structures/mpc_datamodels.py")
    adt = _load("agentlib_mpc.data_structures.admm_datatypes", "data_structures/admm_datatypes.py")
    # known-answer pin from the reference's own test (tests/test_mpc.py:80-86)
    kat = sampling.sample(trajectory=pd.Series([10, 12, 10, 12, 11], index=[0, 10, 20, 30, 40]),
                          grid=[5, 12, 20, 28, 35], current=0)
    assert np.allclose(kat, [11.0, 11.6, 10.0, 11.6, 11.5])
    (OUT / "sampling_golden.json").write_text(json.dumps(sampling_cases(sampling, interp)))
    (OUT / "admm_golden.json").write_text(json.dumps(admm_cases(adt)))
    print("wrote", OUT / "sampling_golden.json", OUT / "admm_golden.json")


if __name__ == "__main__":
    main()
