"""Readers for the on-disk result files the backends and the ADMM fleet write.

Same public functions, argument meaning and return layout as the reference's
`agentlib_mpc/utils/analysis.py` (file:line cited per function), so plotting
and post-processing written against the reference reads MI355X runs unchanged.
Files: backend results (`core/casadi_backend.py:263-307`), ADMM per-iteration
results (`casadi_/admm.py:364-424`), stats files (`mpc_datamodels.py:114-116`).
Host-side pandas only; nothing here touches the device.
"""

import ast
import datetime
import warnings
from pathlib import Path
from typing import Dict, Iterable, Literal, NewType, Optional, Union

import numpy as np
import pandas as pd
from pandas.api.types import is_float_dtype

from agentlib_mpc_amd.data_structures.mpc_datamodels import stats_path

from agentlib_mpc_amd.utils import TIME_CONVERSION, TimeConversionTypes

SimulationTime = NewType("SimulationTime", float)


def _tuple_index(index: pd.Index) -> pd.MultiIndex:
    # results files store the (time, [iteration,] grid time) key as a tuple literal
    return pd.MultiIndex.from_tuples([ast.literal_eval(str(i)) for i in index])


def load_mpc(file: Union[Path, str]) -> pd.DataFrame:
    """Results file -> frame with (time, grid time) rows, (type, name) columns
    (`analysis.py:21-25`)."""
    df = pd.read_csv(file, index_col=[0], header=[0, 1])
    df.index = _tuple_index(df.index)
    return df


def load_admm(file: Union[Path, str]) -> pd.DataFrame:
    """ADMM results file; rows are (time, iteration, grid time) (`analysis.py:17-18`)."""
    return load_mpc(file)


def load_mpc_stats(results_file: Union[str, Path]) -> Optional[pd.DataFrame]:
    """The ``stats_<name>`` file next to a results file, or None if unreadable
    (`analysis.py:28-38`)."""
    try:
        df = pd.read_csv(stats_path(results_file), index_col=0)
    except Exception:
        return None
    if not is_float_dtype(df.index):
        df.index = _tuple_index(df.index)
    return df


def load_sim(file: Path, causality=None) -> pd.DataFrame:
    """Simulator results with a 3-level column header (`analysis.py:41-46`)."""
    df = pd.read_csv(file, header=[0, 1, 2], index_col=0)
    if causality:
        return df[causality].droplevel(level=1, axis=1)
    return df.droplevel(level=2, axis=1).droplevel(level=0, axis=1)


def convert_index(convert_to: Union[TimeConversionTypes, Literal["datetime"]], index: pd.Index):
    """Seconds -> datetime or minutes/hours/days (`analysis.py:61-76`)."""
    if convert_to == "datetime":
        return pd.to_datetime(index.astype(int), unit="s")
    return index / TIME_CONVERSION[convert_to]


def convert_multi_index(data: pd.DataFrame, convert_to: Union[TimeConversionTypes, Literal["datetime"]]):
    """Convert the outer (time) level of a results frame (`analysis.py:49-58`)."""
    outer = convert_index(convert_to, data.index.unique(0))
    return data.set_index(data.index.set_levels(outer, level=0))


def perform_index_update(data: pd.DataFrame, offset: Union[float, Literal["auto"], bool],
                         admm: bool = False) -> pd.DataFrame:
    """Shift the outer time level by ``offset`` ("auto"/True: start at 0; 0/False:
    unchanged) (`analysis.py:79-105`)."""
    if not offset:
        return data
    outer = data.index.get_level_values(0)
    shift = outer[0] if (offset == "auto" or offset is True) else offset
    levels = [outer - shift] + [data.index.get_level_values(k) for k in range(1, 3 if admm else 2)]
    out = data.copy()
    out.index = pd.MultiIndex.from_arrays(levels)
    return out


def _closest(outer: pd.Index, time_step):
    # nearest outer key; ties go to the later key (`analysis.py:144-152`)
    idx = int(np.searchsorted(outer, time_step, side="left"))
    if idx > 0 and (idx == len(outer) or np.fabs(time_step - outer[idx - 1]) < np.fabs(time_step - outer[idx])):
        return outer[idx - 1]
    return outer[idx]


def mpc_at_time_step(data: pd.DataFrame, time_step: float, variable=None, variable_type="variable",
                     index_offset: Union[float, Literal["auto"], bool] = True) -> pd.DataFrame:
    """The prediction made at the step closest to ``time_step``, indexed by
    absolute time (`analysis.py:108-163`)."""
    data = perform_index_update(data, index_offset, admm=False)
    closest = _closest(data.index.get_level_values(0), time_step)
    sel = data[variable_type][variable].loc[closest] if variable else data.loc[closest]
    sel = sel.copy()
    sel.index = sel.index + closest
    return sel


def admm_at_time_step(data: Union[pd.DataFrame, pd.Series], time_step: float = None, variable=None,
                      iteration: float = -1, index_offset: Union[float, Literal["auto"], bool] = True,
                      convert_to: TimeConversionTypes = "seconds") -> pd.DataFrame:
    """One ADMM iteration's prediction at the step closest to ``time_step``;
    negative ``iteration`` counts from the last (`analysis.py:166-241`)."""
    data = convert_multi_index(data, convert_to=convert_to)
    if convert_to != "datetime":
        data = perform_index_update(data, index_offset, admm=True)
    if time_step is None:
        time_step = datetime.datetime.now() if convert_to == "datetime" else 0
    closest = _closest(data.index.get_level_values(0), time_step)
    at_ts = data.loc[closest]
    if iteration < 0:
        iteration = at_ts.index.get_level_values(0).max() + 1 + iteration
    if variable:
        at_it = at_ts.xs(variable, axis=1, level="variable").loc[iteration]
    else:
        at_it = at_ts.loc[iteration]
    at_it = at_it.copy()
    if convert_to == "datetime":
        at_it.index = convert_index(convert_to, at_it.index + closest.value // 1e9)
    else:
        at_it.index = convert_index(convert_to, at_it.index) + closest
    return at_it


def get_number_of_iterations(data: pd.DataFrame) -> Dict[SimulationTime, int]:
    """ADMM iterations performed at each time step (`analysis.py:244-255`)."""
    pairs = data.index.droplevel(2).drop_duplicates()
    counts: Dict[SimulationTime, int] = {}
    for t in pairs.get_level_values(0):
        counts[SimulationTime(t)] = counts.get(SimulationTime(t), 0) + 1
    return counts


def get_time_steps(data: pd.DataFrame) -> Iterable[float]:
    """Sorted time steps at which a solve was recorded (`analysis.py:258-260`)."""
    return sorted(set(data.index.get_level_values(0)))


def _vals_at(data, pick, what):
    vals = pd.Series({t: pick(data.loc[t]) for t in get_time_steps(data)})
    if vals.isna().any():
        warnings.warn(f"Nan detected in {what} values. You may need to select the "
                      "correct column of the DataFrame and drop NaN before.")
    return vals


def first_vals_at_trajectory_index(data: Union[pd.DataFrame, pd.Series]):
    """First entry of each step's trajectory (`analysis.py:263-274`)."""
    return _vals_at(data, lambda d: d.iloc[0], "first")


def last_vals_at_trajectory_index(data: Union[pd.DataFrame, pd.Series]):
    """Last entry of each step's trajectory (`analysis.py:277-290`)."""
    return _vals_at(data, lambda d: d.iloc[-1], "last")
