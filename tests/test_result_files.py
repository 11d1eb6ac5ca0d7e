"""On-disk result formats (CPU): the backend results file + stats file
(`core/casadi_backend.py:263-307`), the ADMM backend's per-iteration results
(`casadi_/admm.py:364-424`) and the coordinator's residual file
(`admm_coordinator.py:437-465`), read back as `utils/analysis.py:21-38` does."""

import ast

import numpy as np
import pandas as pd

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.admm.fleet import ADMMFleet, IterationRecord


def _results(be, cv, now=0.0):
    prob = be.problem
    mi = prob.mpc_inputs(cv, now)
    mi.update(prob.initial_guess(mi))
    p, lbw, ubw, w0 = prob.nlp_inputs(mi)
    stats = {"success": True, "return_status": "Solve_Succeeded", "iter_count": 7, "obj": 1.5}
    return prob.make_results(mi, w0, stats)


def _load_mpc(path):
    df = pd.read_csv(path, header=[0, 1], index_col=0)
    df.index = [ast.literal_eval(i) for i in df.index]
    return df


def test_backend_results_file(tmp_path):
    be, cv = bm.one_room(N=4)
    f = tmp_path / "room.csv"
    be.config.results_file = f
    be.config.save_results = True
    for now in (0.0, 300.0):
        be.save_result_df(_results(be, cv, now), now)
    df = _load_mpc(f)
    assert {i[0] for i in df.index} == {0.0, 300.0}
    assert ("variable", "T") in df.columns and ("parameter", "load") in df.columns
    stats = pd.read_csv(tmp_path / "stats_room.csv", index_col=0)
    assert len(stats) == 2 and stats["iter_count"].tolist() == [7, 7]


def test_admm_backend_iteration_results(tmp_path):
    be, cv = bm.exchange_room(N=4)
    f = tmp_path / "admm.csv"
    be.config.results_file = f
    be.config.save_results = True
    r = _results(be, cv)
    for now, n_it in ((0.0, 3), (120.0, 2)):
        for _ in range(n_it):
            be.save_result_df(r, now)
    # iterations of a step are flushed when the next step starts (`admm.py:405-424`)
    df = _load_mpc(f)
    keys = sorted({i[:2] for i in df.index})
    assert keys == [(0.0, 0), (0.0, 1), (0.0, 2), (120.0, 0)]


def test_coordinator_residual_file(tmp_path):
    recs = [IterationRecord(1.0, 2.0, 0.4, wall_time=0.01), IterationRecord(0.5, 0.25, 0.4, wall_time=0.02)]
    f = tmp_path / "residuals.csv"
    ADMMFleet.save_stats(None, f, 0.0, recs)
    ADMMFleet.save_stats(None, f, 60.0, recs[:1])
    df = pd.read_csv(f, index_col=0)
    assert list(df.columns) == ["primal_residual", "dual_residual", "penalty_parameter", "wall_time"]
    assert [ast.literal_eval(i) for i in df.index] == [(0.0, 0), (0.0, 1), (60.0, 0)]
    np.testing.assert_allclose(df["dual_residual"], [2.0, 0.25, 2.0])


def test_analysis_readers_on_backend_files(tmp_path):
    """`utils/analysis.py` readers on the files the backends write (`analysis.py:17-290`)."""
    from agentlib_mpc_amd.utils import analysis

    be, cv = bm.one_room(N=4)
    f = tmp_path / "room.csv"
    be.config.results_file, be.config.save_results = f, True
    for now in (100.0, 400.0):
        be.save_result_df(_results(be, cv, now), now)
    df = analysis.load_mpc(f)
    assert isinstance(df.index, pd.MultiIndex) and analysis.get_time_steps(df) == [100.0, 400.0]
    st = analysis.load_mpc_stats(f)
    assert st is not None and st["iter_count"].tolist() == [7, 7]
    assert analysis.load_mpc_stats(tmp_path / "missing.csv") is None
    # prediction made at the step closest to t=290 (offset "auto": steps at 0 and 300)
    T = analysis.mpc_at_time_step(df, 290.0, variable="T")
    grid = df["variable"]["T"].loc[400.0]
    np.testing.assert_allclose(T.values, grid.values)
    np.testing.assert_allclose(T.index.values, grid.index.values + 300.0)
    first = analysis.first_vals_at_trajectory_index(df["variable"]["T"])
    np.testing.assert_allclose(first.values, [grid.iloc[0]] * 2)
    last = analysis.last_vals_at_trajectory_index(df["variable"]["T"].dropna())
    assert list(last.index) == [100.0, 400.0]
    hrs = analysis.convert_multi_index(df, "hours")
    np.testing.assert_allclose(sorted(set(hrs.index.get_level_values(0))), [100 / 3600, 400 / 3600])


def test_analysis_readers_on_admm_files(tmp_path):
    from agentlib_mpc_amd.utils import analysis

    be, cv = bm.exchange_room(N=4)
    f = tmp_path / "admm.csv"
    be.config.results_file, be.config.save_results = f, True
    r = _results(be, cv)
    for now, n_it in ((0.0, 3), (120.0, 2), (240.0, 1)):
        for _ in range(n_it):
            be.save_result_df(r, now)
    df = analysis.load_admm(f)
    assert analysis.get_number_of_iterations(df) == {0.0: 3, 120.0: 2, 240.0: 1}
    last_it = analysis.admm_at_time_step(df, time_step=0.0, iteration=-1)
    first_it = analysis.admm_at_time_step(df, time_step=0.0, iteration=0)
    pd.testing.assert_frame_equal(last_it, first_it)
    assert last_it.index[0] == df.loc[(0.0, 2)].index[0]
