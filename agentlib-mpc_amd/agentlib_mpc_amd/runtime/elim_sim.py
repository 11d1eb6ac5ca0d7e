"""Host execution of a generated ``gen_stage_elim`` body (test support).

Translates the straight-line C++ that `stage_elim.emit` produces into Python so
the CPU test suite can check the generated elimination itself -- inertia,
back-substitution operators and Schur blocks -- against dense numpy linear
algebra on the same local matrices, without a GPU.
"""

from __future__ import annotations

import math
import re
from typing import List

import numpy as np


def _fma(a, b, c):
    return a * b + c


def compile_body(lines: List[str]):
    """Compile a generated body; the factor/trailing split line becomes a ``_check``
    that raises when a pivot was singular."""
    out = []
    for ln in lines:
        if ln.strip() == "if (bad) return 1;":
            out.append("if bad:\n    raise _Singular()")
            continue
        s = ln.strip()
        if not s:
            continue
        if s.startswith("//") or s.startswith("__builtin_amdgcn_sched_barrier") or s.startswith("MPCX_ELIM_FENCE"):
            continue
        m = re.match(r"if \((\w+) < 0\.0\) \{ pos \+= 1; neg \+= 1; \} else if \((\w+) \+ (\w+) > 0\.0\) pos \+= 2; "
                     r"else neg \+= 2;", s)
        if m:
            d, a, b = m.groups()
            out.append(f"if {d} < 0.0:\n    pos += 1; neg += 1\nelif {a} + {b} > 0.0:\n    pos += 2\nelse:\n    neg += 2")
            continue
        s = s.replace("const double ", "")
        s = s.replace("!(", "not (").replace("&&", "and")
        s = s.replace("fabs(", "abs(")
        s = s.replace("bad |= ", "bad = bad or ")
        s = s.rstrip(";")
        for part in s.split(";"):
            part = part.strip()
            if part:
                out.append(part)
    return compile("\n".join(out), "<gen_stage_elim>", "exec")


class _Singular(Exception):
    pass


def run(code, F: np.ndarray, ni: int, ntr: int, ns: int, nzx: int):
    env = {"_Singular": _Singular, "F": F, "fma": _fma, "abs": abs, "math": math, "bad": False, "pos": 0, "neg": 0,
           "TR": np.full(ni * ntr, np.nan), "S": np.full(max(ns, 1), np.nan), "ZX": np.full(max(nzx, 1), np.nan),
           "PRM": np.full(ni, -1), "MPCX_N": 1, "MPCX_ELIM_GROWTH": 1e8, "MPCX_RCP": lambda x: 1.0 / x}
    try:
        exec(code, env)
    except _Singular:
        pass
    return dict(bad=bool(env["bad"]), pos=int(env["pos"]), neg=int(env["neg"]), TR=env["TR"], S=env["S"],
                ZX=env["ZX"], PRM=env["PRM"])


def pack(A: np.ndarray) -> np.ndarray:
    """Packed lower triangle (row-major, i*(i+1)/2 + j) of a symmetric matrix."""
    n = A.shape[0]
    return np.concatenate([A[i, :i + 1] for i in range(n)])


def compact(A: np.ndarray, cmap) -> np.ndarray:
    """Compact stage image of a symmetric matrix: entry c holds A[i, j] for the
    ``(i, j)`` of ``GeneratedModel.compact`` (structural nonzeros + fill)."""
    return np.array([A[i, j] for i, j in cmap], dtype=float)
