"""The plugin batch's native attribute reader (csrc/mpcx_pyread.c), CPU only: its columns
against plain getattr, and its read cache (numbers reused while the agent's mapping and the
variable's instance dict are unchanged, by the dicts' version tags) against uncached reads
over random mutation sequences -- every kind of change a caller can make between two calls."""

import copy
import math

import numpy as np
import pytest

from agentlib_mpc_amd.data_structures.mpc_datamodels import MPCVariable
from agentlib_mpc_amd.runtime.native import load_pyread

SPECS = [("T", ("value", "lb", "ub"), True), ("load", ("value",), True), ("u", ("lb", "ub"), False)]


def _fleet(n, seed=0):
    rng = np.random.default_rng(seed)
    return [{"T": MPCVariable("T", float(rng.normal(295, 1)), lb=280.0, ub=310.0),
             "load": MPCVariable("load", float(rng.uniform(0, 200))),
             "u": MPCVariable("u", 0.01, lb=0.0, ub=float(rng.uniform(0.04, 0.06)))} for _ in range(n)]


def _plain(agents):
    cols = []
    for name, attrs, _ in SPECS:
        for a in attrs:
            cols.append([getattr(ag[name], a) for ag in agents])
    return cols


def _read(pr, agents, cache=None):
    ncol = sum(len(a) for _, a, _ in SPECS)
    buf = np.full((ncol, len(agents)), -7.0)
    status, bad = pr.read_columns(agents, SPECS, buf, cache) if cache is not None else \
        pr.read_columns(agents, SPECS, buf)
    return buf, status, bad


@pytest.fixture(scope="module")
def pr():
    try:
        return load_pyread()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"reader not built: {e}")


def test_columns_equal_getattr(pr):
    agents = _fleet(37)
    buf, status, bad = _read(pr, agents)
    assert bad == -1 and not status.strip(b"\x00")
    np.testing.assert_array_equal(buf, np.array(_plain(agents)))


class _Prop(MPCVariable):
    """A subclass whose value is a property (a data descriptor wins over the instance dict)."""

    @property
    def value(self):
        return 1234.5

    @value.setter
    def value(self, v):
        self.__dict__["_v"] = v


def _mutate(rng, agents):
    """One random change of the kinds a caller can make between calls."""
    i = int(rng.integers(len(agents)))
    k = int(rng.integers(9))
    ag = agents[i]
    if k == 0:
        ag["T"].value = float(rng.normal(295, 1))                 # new measurement
    elif k == 1:
        ag["u"].ub = float(rng.uniform(0.04, 0.06))               # new bound
    elif k == 2:
        ag["T"] = MPCVariable("T", float(rng.normal(290, 1)), lb=270.0, ub=300.0)  # new object
    elif k == 3:
        agents[i] = copy.deepcopy(ag)                             # new mapping, same values
        agents[i]["load"].value = float(rng.uniform(0, 200))
    elif k == 4:
        ag["load"].__dict__ = dict(ag["load"].__dict__, value=float(rng.uniform(0, 9)))  # new dict
    elif k == 5:
        v = ag["T"].value
        ag["T"].value = v                                          # same object back: no change
    elif k == 6:
        ag["load"].value = int(rng.integers(0, 100))              # an int
    elif k == 7:
        ag["load"].value = [1.0, 2.0]                             # a trajectory: Python path
    else:
        ag["load"].value = float("nan")                           # NaN: Python path


@pytest.mark.parametrize("seed", range(6))
def test_cached_reads_equal_uncached_reads(pr, seed):
    rng = np.random.default_rng(seed)
    agents = _fleet(23, seed)
    cache = pr.new_cache()
    for step in range(60):
        for _ in range(int(rng.integers(0, 4))):
            _mutate(rng, agents)
        if step % 20 == 19:   # lists / NaN put back to numbers now and then
            for ag in agents:
                v = ag["load"].value
                if not isinstance(v, (int, float)) or (isinstance(v, float) and math.isnan(v)):
                    ag["load"].value = 1.0
        b1, s1, bad1 = _read(pr, agents, cache)
        b2, s2, bad2 = _read(pr, agents)
        assert (s1, bad1) == (s2, bad2)
        ok = np.frombuffer(s1, np.uint8) == 0
        np.testing.assert_array_equal(b1[ok], b2[ok])


def test_cache_sees_class_changes_and_new_batches(pr):
    agents = _fleet(5)
    cache = pr.new_cache()
    _read(pr, agents, cache)
    # a variable object of a class whose value is a property
    p = _Prop("T", 0.0, lb=1.0, ub=2.0)
    agents[2]["T"] = p
    b, _, _ = _read(pr, agents, cache)
    assert b[0, 2] == 1234.5
    # a class changed after the read (a property added): its type version changes
    class Var(MPCVariable):
        pass

    agents[3]["load"] = Var("load", 5.0)
    b, _, _ = _read(pr, agents, cache)
    assert b[3, 3] == 5.0
    Var.value = property(lambda self: -1.0, lambda self, v: None)
    b, _, _ = _read(pr, agents, cache)
    assert b[3, 3] == -1.0
    # another batch size / spec list through the same cache: re-laid out
    fewer = agents[:3]
    b, _, _ = _read(pr, fewer, cache)
    np.testing.assert_array_equal(b, np.array(_plain(fewer)))


def test_missing_variable_raises_key_error_with_cache(pr):
    agents = _fleet(4)
    cache = pr.new_cache()
    _read(pr, agents, cache)
    del agents[1]["load"]
    with pytest.raises(KeyError):
        _read(pr, agents, cache)
    agents[1]["load"] = MPCVariable("load", 3.0)
    b, _, _ = _read(pr, agents, cache)
    assert b[3, 1] == 3.0
