"""Static sparse elimination of a stage interior (generated straight-line code).

The kernel's stage-parallel factorisation eliminates each stage's interior
``A_II`` (stage variables V and the multipliers of the stage rows that are not
bordered) and hands the chain the Schur complement on the trailing rows
``[x_k, c_k]`` plus the back-substitution operators ``W = A_II^{-1} [A_IT | r_I]``
(csrc/mpcx_ipm.hip, ``factor`` / ``stage_tail``).  The generic path is a dense
Bunch-Kaufman factorisation in LDS by a group of lanes: every pivot step
rewrites the whole trailing triangle, so the LDS write pipe and the packed-index
arithmetic bound it.

This module plans the elimination once per model, at code-generation time, from
the structure of the stage KKT matrix:

* every equality row of the interior is paired with a stage variable it touches
  (maximum bipartite matching) and eliminated with it as a 2x2 pivot
  ``[[h, j], [j, -d]]`` -- nonsingular whenever ``j != 0``, inertia (1, 1) when
  ``h d >= 0``, the pivots Bunch-Kaufman would pick on a saddle-point row;
* inequality rows (``-D < 0``) and the remaining variables
  (``H + Sigma + delta_w``) are 1x1 pivots, the variables last so that the
  curvature their rows contribute is in place;
* the order inside each phase is minimum degree on the filled graph.

The generated ``gen_stage_elim`` runs in ONE lane per stage, entirely in
registers: only structural nonzeros and their fill are touched (one_room: 14
interior pivots, ~4x fewer updates than the dense elimination), the trailing
Schur blocks come from sparse dot products against re-read original rows, and
nothing but the outputs is written.  It returns 1 when a pivot is (numerically)
singular -- a fixed variable in a pair, a vanishing Jacobian entry, NaN -- and the
kernel then factors that stage with the dense Bunch-Kaufman path instead, so the
static plan changes only the pivot order, never the result class.  Pivot order
does not change the inertia (Sylvester), which is all the inertia correction
reads.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Sequence, Tuple

ZERO_PIVOT = "1e-20"  # same constant as the kernel's ZERO_PIVOT (dense path)
#: threshold-pivoting bound on the multipliers (Duff-Reid u = 1e-8): a static pivot that is
#: small against its column -- e.g. a variable paired with a row that is open at this stage
#: (MHE stage 0: D ~ 1e16) -- would amplify rounding errors past the inertia test; the
#: stage is then factored densely with Bunch-Kaufman pivoting instead
GROWTH = "MPCX_ELIM_GROWTH"  # 1e8 unless the build defines it (diagnostics)
#: scheduling fence between pivot blocks / substitution sweeps: keeps the live set (and the
#: callee-saved VGPRs the non-inlined caller would have to spill) small
SCHED = "  MPCX_ELIM_FENCE;"  # __builtin_amdgcn_sched_barrier(0) unless overridden (codegen.py)
#: line between the factor and trailing parts: a singular pivot returns before any output
CHECK = "  if (bad) return 1;"


@dataclasses.dataclass
class ElimPlan:
    blocks: List[Tuple[int, ...]]     # pivot blocks in elimination order (local indices)
    cols: List[List[int]]             # per block: remaining interior neighbours (filled graph)
    n_update: int                     # entry updates of the interior elimination
    nnz_l: int                        # off-diagonal multiplier entries (per pivot index)
    flops: int = 0                    # FP64 operations of the generated body (fma = 2)


def count_flops(lines: Sequence[str]) -> int:
    """FP64 operations of generated straight-line code: fma counts 2, every other
    arithmetic operator outside index brackets 1 (comparisons are not counted)."""
    import re

    n = 0
    for ln in lines:
        s = ln.strip()
        if s.startswith("//") or s.startswith("__builtin") or s.startswith("MPCX_ELIM_FENCE") or s.startswith("bad |=") or s.startswith("if ("):
            continue
        if "=" not in s:
            continue
        rhs = s.split("=", 1)[1]
        rhs = re.sub(r"\[[^\]]*\]", "", rhs)      # drop index expressions
        n += 2 * rhs.count("fma(")
        n += len(re.findall(r"(?<=[\w)\s])\s*[-+*/]\s*(?=[\w(])", rhs))
    return n


def _match(rows: List[List[int]], n_cols: int) -> List[int]:
    """Maximum bipartite matching rows -> columns (augmenting paths, columns in order)."""
    match_col = [-1] * n_cols

    def augment(r, seen):
        for c in rows[r]:
            if c in seen:
                continue
            seen.add(c)
            if match_col[c] < 0 or augment(match_col[c], seen):
                match_col[c] = r
                return True
        return False

    for r in range(len(rows)):
        augment(r, set())
    return match_col


def _weighted_match(eq_duals, nv, g, weight):
    """Pairs (variable -> equality row) maximising the summed entry weights among the
    maximum matchings (Hungarian method); None if scipy is unavailable."""
    try:
        import numpy as np
        from scipy.optimize import linear_sum_assignment
    except ImportError:  # pragma: no cover
        return None
    big = 1e6
    C = np.full((len(eq_duals), nv), big)
    for a, r in enumerate(eq_duals):
        for c in g[r]:
            if c < nv:
                C[a, c] = -weight.get((r, c), 1.0)
    ri, ci = linear_sum_assignment(C)
    return {int(c): eq_duals[int(a)] for a, c in zip(ri, ci) if C[a, c] < big}


def plan(adj: Sequence[set], ni: int, nv: int, eq_duals: Sequence[int], weight=None) -> ElimPlan:
    """Elimination plan for the interior ``0..ni-1`` of a local system whose
    symmetric off-diagonal structure is ``adj`` (indices >= ni are trailing rows:
    they receive fill but never pivot).  ``eq_duals``: interior dual indices
    (nv <= i < ni) of equality rows; ``weight[(row, var)]``: preference of a pairing
    (constant Jacobian entries of magnitude >= 1 never vanish; a state-dependent entry,
    e.g. a network derivative, can be small at the iterate and make the 2x2 pivot
    nearly singular)."""
    g = [set(a) for a in adj]
    rows = [sorted(c for c in g[r] if c < nv) for r in eq_duals]
    mc = _match(rows, nv)
    pairs = {}
    for v, r in enumerate(mc):
        if r >= 0:
            pairs[v] = eq_duals[r]
    if weight:
        wp = _weighted_match(eq_duals, nv, g, weight)
        if wp is not None and len(wp) == len(pairs):
            pairs = wp
    paired = set(pairs) | set(pairs.values())
    phase1 = [(v, d) for v, d in pairs.items()] + [(i,) for i in range(nv, ni) if i not in paired]
    phase2 = [(i,) for i in range(nv) if i not in paired]
    alive = set(range(len(g)))
    blocks, cols, n_update = [], [], 0
    for phase in (phase1, phase2):
        todo = list(phase)
        while todo:
            def ext(b):
                nb = set().union(*(g[i] for i in b)) & alive
                return len(nb - set(b))
            b = min(todo, key=lambda b: (ext(b), b[0]))
            todo.remove(b)
            nb = sorted((set().union(*(g[i] for i in b)) & alive) - set(b))
            for i in b:
                alive.discard(i)
            for i in nb:  # fill: the neighbours form a clique
                g[i].update(j for j in nb if j != i)
            inner = [i for i in nb if i < ni]
            n_update += len(inner) * (len(inner) + 1) // 2
            blocks.append(tuple(b))
            cols.append(inner)
    nnz_l = sum(len(c) * len(b) for b, c in zip(blocks, cols))
    return ElimPlan(blocks, cols, n_update, nnz_l)


def emit(P: Sequence[Sequence[bool]], ni: int, nv: int, nx: int, nc: int,
         eq_duals: Sequence[int], weight=None) -> Tuple[List[str], List[str], ElimPlan]:
    """C++ of ``gen_stage_elim`` for a local system with structure ``P`` ((nloc+1)^2,
    symmetric, border row last; trailing rows x_k = ni..ni+nx-1, c_k = ni+nx..ni+nx+nc-1,
    border = ni+nx+nc), as two parts:

    * factor: in-place sparse block LDL^T of the interior in the packed LDS image ``F``
      (multipliers over the eliminated entries, pivot-block inverses on the diagonal);
      only the pivot column of the current block is held in registers;
    * trailing: per trailing column t, ``w_t = A_II^{-1} a_t`` by sparse forward /
      block-diagonal / backward substitution (``TR``), then the Schur entries of the
      rows already solved against the untouched trailing rows of ``F`` (``S``, ``ZX``).

    The caller returns between the two parts when a pivot was singular (``bad``); the
    image is then re-assembled for the dense path."""
    n = len(P)
    ntr = nx + nc + 1
    assert n == ni + ntr
    adj = [set(j for j in range(n) if j != i and (P[i][j] or P[j][i])) for i in range(n)]
    pl = plan(adj, ni, nv, eq_duals, weight)

    def pk(i, j):
        i, j = max(i, j), min(i, j)
        return i * (i + 1) // 2 + j

    fac: List[str] = []
    cnt = [0]

    def new(out: List[str], expr: str) -> str:
        cnt[0] += 1
        name = f"e{cnt[0]}"
        out.append(f"  const double {name} = {expr};")
        return name

    # ---- factor: in place, interior entries only ----
    for bi, (b, col) in enumerate(zip(pl.blocks, pl.cols)):
        fac.append(f"  // pivot block {bi}: {list(b)}, column {col}")
        fac.append(SCHED)
        if len(b) == 1:
            p = b[0]
            d = new(fac, f"F[{pk(p, p)}]")
            fac.append(f"  bad |= !(fabs({d}) > {ZERO_PIVOT}); pos += {d} > 0.0; neg += {d} < 0.0;")
            r = new(fac, f"MPCX_RCP({d})")
            u = {i: new(fac, f"F[{pk(i, p)}]") for i in col}
            lm = {i: (new(fac, f"{u[i]} * {r}"),) for i in col}
            if col:
                fac.append(f"  bad |= !(" + " && ".join(f"fabs({lm[i][0]}) <= {GROWTH}" for i in col) + ");")
            for x, i in enumerate(col):
                for j in col[:x + 1]:
                    fac.append(f"  F[{pk(i, j)}] = fma(-{lm[i][0]}, {u[j]}, F[{pk(i, j)}]);")
            fac.append(f"  F[{pk(p, p)}] = {r};")
            for i in col:
                fac.append(f"  F[{pk(i, p)}] = {lm[i][0]};")
        else:
            p, q = b
            a11, a21, a22 = new(fac, f"F[{pk(p, p)}]"), new(fac, f"F[{pk(q, p)}]"), new(fac, f"F[{pk(q, q)}]")
            det = new(fac, f"{a11} * {a22} - {a21} * {a21}")
            fac.append(f"  bad |= !(fabs({det}) > {ZERO_PIVOT} * {ZERO_PIVOT});")
            fac.append(f"  if ({det} < 0.0) {{ pos += 1; neg += 1; }} else if ({a11} + {a22} > 0.0) pos += 2; "
                       f"else neg += 2;")
            rd = new(fac, f"MPCX_RCP({det})")
            u1 = {i: new(fac, f"F[{pk(i, p)}]") for i in col}
            u2 = {i: new(fac, f"F[{pk(i, q)}]") for i in col}
            lm = {i: (new(fac, f"({u1[i]} * {a22} - {u2[i]} * {a21}) * {rd}"),
                      new(fac, f"({u2[i]} * {a11} - {u1[i]} * {a21}) * {rd}")) for i in col}
            if col:
                fac.append(f"  bad |= !(" + " && ".join(f"fabs({lm[i][0]}) <= {GROWTH} && fabs({lm[i][1]}) <= {GROWTH}"
                                                       for i in col) + ");")
            for x, i in enumerate(col):
                for j in col[:x + 1]:
                    fac.append(f"  F[{pk(i, j)}] = fma(-{lm[i][0]}, {u1[j]}, fma(-{lm[i][1]}, {u2[j]}, F[{pk(i, j)}]));")
            fac.append(f"  F[{pk(p, p)}] = {a22} * {rd}; F[{pk(q, p)}] = -{a21} * {rd}; F[{pk(q, q)}] = {a11} * {rd};")
            for i in col:
                fac.append(f"  F[{pk(i, p)}] = {lm[i][0]}; F[{pk(i, q)}] = {lm[i][1]};")

    # ---- trailing columns ----
    tra: List[str] = []

    def orig(i, j):  # original (assembled) entry of a trailing row: untouched by the factor part
        return f"F[{pk(i, j)}]" if (P[i][j] or P[j][i] or i == j) else None

    def schur_dot(t1, w):  # sum_p a_t1[p] w[p] over the structural nonzeros of row t1
        terms = [f"{orig(t1, p)} * {w[p]}" for p in range(ni) if orig(t1, p) is not None and w[p] != "0.0"]
        return " + ".join(terms) if terms else "0.0"

    # Schur entries wanted, by column: S00 (x_k x x_k), S11 (c_k x c_k), S10 (c_k x x_k), zx
    nxx, ncc = max(nx, 1) ** 2, max(nc, 1) ** 2
    want: Dict[int, List[Tuple[int, str]]] = {}

    def add(ri, ci, dest):
        want.setdefault(max(ri, ci), []).append((min(ri, ci), dest))

    for e in range(nx * nx):
        add(ni + e // nx, ni + e % nx, f"S[{e}]")
    for f in range(nc * nc):
        add(ni + nx + f // nc, ni + nx + f % nc, f"S[{nxx + f}]")
    for f in range(nc * nx):
        add(ni + nx + f // nx, ni + f % nx, f"S[{nxx + ncc + f}]")
    for c in range(nx + nc):
        add(n - 1, ni + c, f"ZX[{c}]")
    for t in range(ntr):
        ti = ni + t
        tra.append(f"  // trailing column {t} (local {ti})")
        tra.append(SCHED)
        y: Dict[int, str] = {p: orig(ti, p) for p in range(ni) if orig(ti, p) is not None}
        for bi, b in enumerate(pl.blocks):  # forward: L y = a_t
            if not any(p in y for p in b):
                continue
            if len(b) == 1 and b[0] in y and y[b[0]].startswith("F["):
                y[b[0]] = new(tra, y[b[0]])
            for i in pl.cols[bi]:
                term = " + ".join(f"F[{pk(i, p)}] * {y[p]}" for p in b if p in y)
                y[i] = new(tra, f"{y[i]} - ({term})" if i in y else f"-({term})")
        z: Dict[int, str] = {}
        for bi, b in enumerate(pl.blocks):  # z = D^-1 y (inverses stored on the diagonal)
            if len(b) == 1:
                z[b[0]] = new(tra, f"{y[b[0]]} * F[{pk(b[0], b[0])}]") if b[0] in y else "0.0"
            else:
                p, q = b
                y1, y2 = y.get(p), y.get(q)
                if y1 is None and y2 is None:
                    z[p] = z[q] = "0.0"
                    continue
                y1, y2 = y1 or "0.0", y2 or "0.0"
                z[p] = new(tra, f"F[{pk(p, p)}] * {y1} + F[{pk(q, p)}] * {y2}")
                z[q] = new(tra, f"F[{pk(q, p)}] * {y1} + F[{pk(q, q)}] * {y2}")
        w: Dict[int, str] = {}
        tra.append(SCHED)
        for bi in range(len(pl.blocks) - 1, -1, -1):  # backward: L^T w = z
            b = pl.blocks[bi]
            for p in b:
                terms = [f"F[{pk(i, p)}] * {w[i]}" for i in pl.cols[bi] if w[i] != "0.0"]
                w[p] = new(tra, f"{z[p]} - ({' + '.join(terms)})") if terms else z[p]
        for p in range(ni):
            tra.append(f"  TR[{t * ni + p} * MPCX_N] = {w[p]};")  # stage-minor in HBM
        for ri, dest in want.get(ti, []):  # value(ri, ti) = A[ri][ti] - a_ri . w_ti
            tra.append(f"  {dest} = {orig(ri, ti) or '0.0'} - ({schur_dot(ri, w)});")
    pl.flops = count_flops(fac) + count_flops(tra)
    return fac, tra, pl
