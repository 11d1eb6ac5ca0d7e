"""Read the MI355X backends' result files with the REFERENCE's own readers.

Run in the build container only (needs /root/reference; never on the GPU box):

    python tests/golden/make_reader_goldens.py

The product writers (`tests/result_file_cases.py`) write results, stats and residual files;
these are copied to `tests/golden/result_files/` (fixture inputs) and read by
`agentlib_mpc/utils/analysis.py` (``load_mpc``, ``load_mpc_stats``, ``load_admm``,
``get_number_of_iterations``, ``admm_at_time_step``, ``mpc_at_time_step``,
``first_vals_at_trajectory_index``, ``last_vals_at_trajectory_index``,
``convert_multi_index``) and `utils/plotting/admm_residuals.py` (``load_residuals``),
executed with stubbed package roots as in `make_golden.py`.  Only the readers' outputs are
written (`reader_golden.json`); no reference source is copied.
"""

from __future__ import annotations

import json
import math
import os
import pathlib
import shutil
import sys
import tempfile
import types

ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT), str(ROOT / "agentlib-mpc_amd")]

from tests.golden.make_golden import REF, _load, _stub_packages  # noqa: E402

OUT = pathlib.Path(__file__).resolve().parent


def _load_reference_readers():
    _stub_packages()
    utils = sys.modules["agentlib_mpc.utils"]
    exec(compile((REF / "utils" / "__init__.py").read_text(), str(REF / "utils" / "__init__.py"), "exec"),
         utils.__dict__)
    _load("agentlib_mpc.data_structures.interpolation", "data_structures/interpolation.py")
    _load("agentlib_mpc.data_structures.coordinator_datatypes", "data_structures/coordinator_datatypes.py")
    _load("agentlib_mpc.data_structures.mpc_datamodels", "data_structures/mpc_datamodels.py")
    analysis = _load("agentlib_mpc.utils.analysis", "utils/analysis.py")
    plotting = types.ModuleType("agentlib_mpc.utils.plotting")
    plotting.__path__ = [str(REF / "utils" / "plotting")]
    sys.modules["agentlib_mpc.utils.plotting"] = plotting
    basic = types.ModuleType("agentlib_mpc.utils.plotting.basic")  # matplotlib styling only
    basic.Style = basic.make_fig = basic.make_grid = basic.EBCColors = None
    sys.modules["agentlib_mpc.utils.plotting.basic"] = basic
    residuals = _load("agentlib_mpc.utils.plotting.admm_residuals", "utils/plotting/admm_residuals.py")
    return analysis, residuals


def _j(x):
    """JSON-able copy (NaN -> None, tuples -> lists)."""
    import numpy as np
    import pandas as pd

    if isinstance(x, pd.DataFrame):
        return {"index": _j(list(x.index)), "columns": _j([list(c) if isinstance(c, tuple) else c for c in x.columns]),
                "values": _j(x.to_numpy().tolist())}
    if isinstance(x, pd.Series):
        return {"index": _j(list(x.index)), "values": _j(x.to_numpy().tolist())}
    if isinstance(x, dict):
        return {str(k): _j(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_j(v) for v in x]
    if isinstance(x, (np.floating, float)):
        return None if math.isnan(float(x)) else float(x)
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.bool_,)):
        return bool(x)
    return x


def main():
    from tests import result_file_cases as rfc

    analysis, residuals = _load_reference_readers()
    with tempfile.TemporaryDirectory() as tmp:
        d = rfc.write_all(tmp)
        dst = OUT / "result_files"
        for rel in rfc.FILES:
            (dst / rel).parent.mkdir(parents=True, exist_ok=True)
            shutil.copyfile(d / rel, dst / rel)
        mpc = analysis.load_mpc(d / "mpc" / "room.csv")
        admm = analysis.load_admm(d / "admm" / "admm.csv")
        out = {
            "load_mpc": _j(mpc),
            "load_mpc_stats": _j(analysis.load_mpc_stats(d / "mpc" / "room.csv")),
            "get_time_steps_mpc": _j(list(analysis.get_time_steps(mpc))),
            "mpc_at_time_step_T_290": _j(analysis.mpc_at_time_step(mpc, 290.0, variable="T")),
            "first_vals_T": _j(analysis.first_vals_at_trajectory_index(mpc["variable"]["T"])),
            "last_vals_T": _j(analysis.last_vals_at_trajectory_index(mpc["variable"]["T"].dropna())),
            "convert_multi_index_hours": _j(list(analysis.convert_multi_index(mpc.copy(), "hours").index)),
            "load_admm_index": _j(list(admm.index)),
            "load_admm_stats": _j(analysis.load_mpc_stats(d / "admm" / "admm.csv")),
            "get_number_of_iterations": _j(analysis.get_number_of_iterations(admm)),
            "admm_at_time_step_0_last": _j(analysis.admm_at_time_step(admm, time_step=0.0, iteration=-1)),
            "load_residuals": _j(residuals.load_residuals(d / "residuals.csv")),
        }
    (OUT / "reader_golden.json").write_text(json.dumps(out, indent=1))
    print(OUT / "reader_golden.json")


if __name__ == "__main__":
    main()
