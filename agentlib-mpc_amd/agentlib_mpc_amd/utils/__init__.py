"""Host-side utilities: time units (`agentlib_mpc/utils/__init__.py:7-27`),
trajectory sampling (`sampling.py`) and result-file readers (`analysis.py`)."""

from typing import Dict, List, Literal, Tuple

TimeConversionTypes = Literal["seconds", "minutes", "hours", "days"]
TIME_CONVERSION: Dict[str, int] = {"seconds": 1, "minutes": 60, "hours": 3600, "days": 86400}


def is_time_in_intervals(time: float, intervals: List[Tuple[float, float]]) -> bool:
    """True if ``time`` lies in any closed interval ``(start, end)``."""
    return any(lo <= time <= hi for lo, hi in intervals)
