"""Host-side utilities: time units (`agentlib_mpc/utils/__init__.py:7-27`) and
trajectory sampling (`sampling.py`).  Result files are read with the reference's own
readers (`agentlib_mpc/utils/analysis.py`); `tests/golden/make_reader_goldens.py` pins
that they parse this package's files."""

from typing import Dict, List, Literal, Tuple

TimeConversionTypes = Literal["seconds", "minutes", "hours", "days"]
TIME_CONVERSION: Dict[str, int] = {"seconds": 1, "minutes": 60, "hours": 3600, "days": 86400}


def is_time_in_intervals(time: float, intervals: List[Tuple[float, float]]) -> bool:
    """True if ``time`` lies in any closed interval ``(start, end)``."""
    return any(lo <= time <= hi for lo, hi in intervals)
