"""Generate the per-model HIP source of the batched interior-point kernel.

The reference lets CasADi expand the NLP into straight-line SX code and
evaluates it through its VM inside IPOPT callbacks
(`agentlib_mpc/data_structures/casadi_utils.py:191-217`, ``expand=True``;
Windows-only C code generation at :313-369).  Here the generic stage
function of a :class:`StageNLP` (one stage of the transcription, see
`optimization_backends/discretization.py`) is differentiated symbolically and
emitted as four ``__device__`` functions:

* ``gen_stage_fg``      cost and constraint residuals (line search),
* ``gen_stage_bounds``  constraint bounds (may depend on parameters),
* ``gen_stage_gj``      cost gradient and dense constraint Jacobian,
* ``gen_stage_hess``    Hessian of the stage Lagrangian ``σ f + λᵀ g``.

``gen_stage_gj`` and ``gen_stage_hess`` also write their entries straight
into ``lp``, the packed lower triangle of the stage's local KKT system in the
kernel's local order ``[V, λ, x_k, x_{k+1}, rhs]`` (Jacobian rows scaled by
the constraint scaling ``G[r]``), so the factorisation assembles a stage by a
contiguous copy instead of gathering strided derivative entries.

The file ends by including the generic kernel `csrc/mpcx_ipm.hip`, so each
model gets one fully specialised code object (all dimensions compile-time).
"""

from __future__ import annotations

import dataclasses
import hashlib
import re
from typing import Dict, List

from agentlib_mpc_amd import symbolic as sx
from agentlib_mpc_amd.runtime import stage_elim
from agentlib_mpc_amd.optimization_backends.discretization import StageNLP

KERNEL_ABI_VERSION = 8  # must equal MPCX_KERNEL_ABI (csrc/mpcx_internal.h)


@dataclasses.dataclass
class GeneratedModel:
    source: str
    key: str
    dims: Dict[str, int]
    flops: Dict[str, int]
    nnz: Dict[str, int]
    #: built with MPCX_FORCE_BLOCK_CHAIN (stage interiors singular even with bordered rows)
    block_chain_only: bool = False
    #: stage rows kept in the border (their multipliers are chained with x_{k+1})
    bordered_rows: list = dataclasses.field(default_factory=list)
    #: static elimination plan of the stage interior and its generated body (stage_elim.py)
    elim: object = None
    elim_lines: list = dataclasses.field(default_factory=list)
    #: plan of stage 0 when rows that are equalities at k >= 1 are open there (else None)
    elim0: object = None
    elim0_lines: list = dataclasses.field(default_factory=list)
    pattern: list = dataclasses.field(default_factory=list)
    #: compact stage image: (row, column) of each stored entry (lp, LDS image, elimination)
    compact: list = dataclasses.field(default_factory=list)
    #: local index of each stage row in the stage system
    crow: list = dataclasses.field(default_factory=list)


def _bindings(nlp: StageNLP) -> Dict[sx.Expr, str]:
    st = nlp.stage
    b: Dict[sx.Expr, str] = {}
    for i, s in enumerate(st.local):
        b[s] = f"L[{i}]"
    for i, s in enumerate(st.PS):
        b[s] = f"PS[{i}]"
    for i, s in enumerate(st.PG):
        b[s] = f"PG[{i}]"
    b[st.TK] = "TK"
    return b


def _structural_rank(rows: List[set], n_cols: int) -> int:
    """Maximum bipartite matching of equality rows to the stage variables they touch."""
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

    return sum(1 for r in range(len(rows)) if augment(r, set()))


def equality_rows(nlp: StageNLP, stage: int = None):
    """Stage rows whose bound expressions coincide at a random parameter point, at an
    inner stage (k >= 1) or at ``stage``."""
    import numpy as np

    st = nlp.stage
    rng = np.random.default_rng(0)
    vals = {s: float(rng.uniform(0.5, 1.5)) for s in list(st.PS) + list(st.PG)}
    vals[st.TK] = nlp.ts * (min(1, nlp.N - 1) if stage is None else stage)
    lb = np.array(sx.evaluate(st.g_lb, vals), float)
    ub = np.array(sx.evaluate(st.g_ub, vals), float)
    return [int(i) for i in np.flatnonzero(lb == ub)]


def interior_rank_deficient(nlp: StageNLP, bordered=()) -> bool:
    """True when the equality rows of a stage (except the ``bordered`` ones) cannot all be
    matched to the stage's own variables V (structural rank of their V-Jacobian below the
    row count), e.g. more states than free inputs per interval (continuity rows), a
    carried previous control, or an MHE link row.  The kernel's stage-parallel
    elimination needs nonsingular stage interiors; near-singular ones are not always
    caught by its zero-pivot test and give inaccurate Newton steps.  Equality rows are
    those whose bound expressions coincide at a random parameter point."""
    st = nlp.stage
    if not st.g or not st.V:
        return False
    col = {v.uid: i for i, v in enumerate(st.V)}
    rows = []
    skip = set(bordered)
    for i in equality_rows(nlp):
        if int(i) in skip:
            continue
        rows.append({col[f.uid] for f in sx.free_symbols([st.g[i]]) if f.uid in col})
    return _structural_rank(rows, len(st.V)) < len(rows)


def continuity_rows(nlp: StageNLP) -> list:
    """Stage rows through x_{k+1} (the continuity / shift equations)."""
    st = nlp.stage
    x1 = {v.uid for v in st.X1}
    return [r for r, g in enumerate(st.g) if any(f.uid in x1 for f in sx.free_symbols([g]))]


def factorisation_plan(nlp: StageNLP):
    """(bordered rows, block chain only): the kernel eliminates every stage interior in
    parallel; when the interior would be singular with the continuity rows in it (more
    states than free stage inputs: MHE lifts, change penalties, 2-state zone models) those
    rows are kept in the border and their multipliers join x_{k+1} in the chain; only if
    that still leaves the interior singular is the sequential block chain used."""
    if not (nlp.force_block_chain or interior_rank_deficient(nlp)):
        return [], False
    cont = continuity_rows(nlp)
    if nlp.nx > 0 and len(cont) == nlp.nx and not interior_rank_deficient(nlp, cont):
        return cont, False
    return [], True


def _network_section(nlp: StageNLP, bind, fg_assign, gj_all, h_all, emit_gj, emit_h, to_compact):
    """Device code of the network evaluations on the FP64 matrix cores (empty when the
    stage has no network node): ``gen_stage_netin`` (one lane per stage writes the inputs
    of every call site to LDS), ``gen_net_{fg,gj,hess}`` (the wave evaluates each network
    over all stages x call sites, ``mpcx_net::eval``, csrc/mpcx_net_mfma.h) and the stage
    functions ``gen_stage_{fg,gj,hess}_m`` that read the network entries from LDS instead
    of looping over the hidden units.  Returns (lines, defines, X doubles, output doubles)."""
    sites = {}
    for outs in (fg_assign, gj_all, h_all):
        for key, val in sx.network_sites([e for _, e in outs]).items():
            sites.setdefault(key, val)
    if not sites:
        return [], [], 0, 0
    N = nlp.N
    nets: Dict[int, list] = {}
    for key in sites:
        nets.setdefault(key[0], []).append(key)
    sidx = {key: q for keys in nets.values() for q, key in enumerate(keys)}
    xoff, netx = {}, 0
    for nid, keys in nets.items():
        xoff[nid] = netx
        netx += N * len(keys) * sx.network(nid).n_in

    def layout(outs):
        mem = {nid: set() for nid in nets}
        for (nid, _), (_, _, members) in sx.network_sites([e for _, e in outs]).items():
            mem[nid].update(members)
        lay, o = {}, 0
        for nid, keys in nets.items():
            m, R = mem[nid], N * len(keys)
            wv = ("v", -1, -1) in m
            d1 = sorted(i for (k, i, _) in m if k == "d")
            d2 = sorted((i, j) for (k, i, j) in m if k == "dd")
            ov = o
            og = ov + (R if wv else 0)
            oh = og + R * len(d1)
            o = oh + R * len(d2)
            lay[nid] = dict(wv=wv, d1=d1, d2=d2, R=R, ov=ov, og=og, oh=oh)
        return lay, o

    def reader(lay):
        def read(nid, key, mk):
            q, Q, L = sidx[(nid, key)], len(nets[nid]), lay[nid]
            row = f"(K * {Q} + {q})"
            if mk[0] == "v":
                return f"NO[{L['ov']} + {row}]"
            if mk[0] == "d":
                return f"NO[{L['og']} + {row} * {len(L['d1'])} + {L['d1'].index(mk[1])}]"
            return f"NO[{L['oh']} + {row} * {len(L['d2'])} + {L['d2'].index((mk[1], mk[2]))}]"
        return read

    kinds = {"fg": layout(fg_assign), "gj": layout(gj_all), "hess": layout(h_all)}
    neto = max(o for _, o in kinds.values())
    lines: List[str] = ['#include "mpcx_net_mfma.h"']
    for kind, (lay, _) in kinds.items():
        for nid, L in lay.items():
            net = sx.network(nid)
            if L["d1"]:
                lines.append(f"__constant__ int ANN{nid}_D1{kind}[{len(L['d1'])}] = {{{', '.join(map(str, L['d1']))}}};")
            if L["d2"]:
                pw = [net.W1[a, j] * net.W1[b, j] for a, b in L["d2"] for j in range(net.H)]
                lines.append(f"__constant__ double ANN{nid}_PW{kind}[{len(pw)}] = "
                             f"{{{', '.join(sx._c_literal(float(v)) for v in pw)}}};")
    sig = "const double* __restrict__ L, const double* __restrict__ PS, const double* __restrict__ PG, const double TK"
    xa = []
    for (nid, key), (_, args, _) in sites.items():
        nin = sx.network(nid).n_in
        xa += [(f"X[{xoff[nid]} + (K * {len(nets[nid])} + {sidx[(nid, key)]}) * {nin} + {i}]", a)
               for i, a in enumerate(args)]
    lines += [f"__device__ __forceinline__ void gen_stage_netin({sig}, double* __restrict__ X, const int K) {{",
              *sx.CodeGen(bind, prefix="n").emit(xa), "}"]
    for kind, (lay, _) in kinds.items():
        lines.append(f"__device__ __forceinline__ void gen_net_{kind}(const mpcx_elim_ld* X, mpcx_elim_ld* O, "
                     f"const int lane) {{")
        for nid, L in lay.items():
            if not (L["wv"] or L["d1"] or L["d2"]):
                continue
            net = sx.network(nid)
            d1 = f"ANN{nid}_D1{kind}" if L["d1"] else "nullptr"
            pw = f"ANN{nid}_PW{kind}" if L["d2"] else "nullptr"
            lines.append(f"  mpcx_net::eval<{L['R']}, {net.n_in}, {net.H}, {sx.ACT_CODE[net.act]}, "
                         f"{'true' if L['wv'] else 'false'}, {len(L['d1'])}, {len(L['d2'])}>("
                         f"X + {xoff[nid]}, O + {L['ov']}, O + {L['og']}, O + {L['oh']}, ANN{nid}_W1T, ANN{nid}_B1, "
                         f"ANN{nid}_W2, {sx._c_literal(net.b2)}, {d1}, {pw}, lane);")
        lines.append("}")
    ext = "const double* __restrict__ NO, const int K"
    lines += [f"__device__ __forceinline__ void gen_stage_fg_m({sig}, double* __restrict__ f, double* __restrict__ g, "
              f"const int S, {ext}) {{",
              *sx.CodeGen(bind, prefix="a", net_lds=reader(kinds["fg"][0])).emit(fg_assign), "}",
              f"__device__ __forceinline__ void gen_stage_gj_m({sig}, double* __restrict__ grad, double* __restrict__ jac, "
              f"const int S, const double* __restrict__ G, double* __restrict__ lp, const double* __restrict__ LM, "
              f"double* __restrict__ jtl, const int full, {ext}) {{",
              *to_compact(emit_gj(reader(kinds["gj"][0])), "lp"), "}",
              f"__device__ __forceinline__ void gen_stage_hess_m({sig}, const double sigma, const double* __restrict__ lam, "
              f"double* __restrict__ hess, const int S, double* __restrict__ lp, const int full, {ext}) {{",
              *to_compact(emit_h(reader(kinds["hess"][0])), "lp"), "}"]
    defs = ["#define MPCX_NET_MFMA 1", f"#define MPCX_NETX {netx}", f"#define MPCX_NETO {max(neto, 1)}"]
    return lines, defs, netx, max(neto, 1)


def generate(nlp: StageNLP, ts: float = None, _bordered=None) -> GeneratedModel:
    st = nlp.stage
    if _bordered is None:
        bordered, force_chain = factorisation_plan(nlp)
    else:
        bordered, force_chain = list(_bordered), False
    loc = st.local
    nl = len(loc)
    ng = nlp.ng
    bind = _bindings(nlp)
    sigma = sx.sym("sigma")
    lam = [sx.sym(f"lam[{i}]") for i in range(ng)]
    hb = dict(bind)
    hb[sigma] = "sigma"
    for i, s in enumerate(lam):
        hb[s] = f"lam[{i}]"

    grad = sx.gradient(st.cost, loc)
    jac = sx.jacobian(st.g, loc)
    lag = sx.add(sx.mul(sigma, st.cost), sx.sum1(sx.mul(l, g) for l, g in zip(lam, st.g)))
    lgrad = sx.gradient(lag, loc)
    hess = [[sx.diff(lgrad[i], loc[j]) for j in range(nl)] for i in range(nl)]

    # -- fg --
    fg_assign = [("f[0]", st.cost)] + [(f"g[{i} * S]", e) for i, e in enumerate(st.g)]
    fg_lines = sx.CodeGen(bind, prefix="a").emit(fg_assign)
    # -- bounds (parameters only) --
    for e in st.g_lb + st.g_ub:
        if any(s.uid in {v.uid for v in loc} for s in sx.free_symbols([e])):
            raise ValueError("constraint bounds must not depend on optimization variables")
    cg = sx.CodeGen(bind, prefix="b")
    bd_lines = cg.emit([(f"lb[{i} * S]", e) for i, e in enumerate(st.g_lb)]
                       + [(f"ub[{i} * S]", e) for i, e in enumerate(st.g_ub)])
    # local order of the kernel's stage system:
    #   [V (nv), lambda_rest (ng - nmu), x_k (nx), mu_k (nmu), x_{k+1} (nx), rhs]
    nx, nv = nlp.nx, nlp.nv
    nmu = len(bordered)
    ni = nv + ng - nmu
    rest = [r for r in range(ng) if r not in set(bordered)]
    crow = [0] * ng
    for q, r in enumerate(rest):
        crow[r] = nv + q
    for q, r in enumerate(bordered):
        crow[r] = ni + nx + q
    nloc = ni + 2 * nx + nmu
    lrow = [-1] * (nloc + 1)
    for r, li in enumerate(crow):
        lrow[li] = r

    def lidx(n: int) -> int:
        if n < nx:
            return ni + n
        if n < nx + nv:
            return n - nx
        return ni + nx + nmu + (n - nx - nv)

    def pk(i: int, j: int) -> int:
        i, j = max(i, j), min(i, j)
        return i * (i + 1) // 2 + j

    # -- gradient + jacobian (structural zeros are never written) --
    g_assign = [(f"grad[{j} * S]", e) for j, e in enumerate(grad) if not e.is_const(0.0)]
    j_assign = [(f"jac[{i * nl + j} * S]", jac[i][j]) for i in range(ng) for j in range(nl)
                if not jac[i][j].is_const(0.0)]
    gj_assign = g_assign + j_assign
    gsym = [sx.sym(f"G[{r}]") for r in range(ng)]
    lmsym = [sx.sym(f"LM[{r}]") for r in range(ng)]
    gb = dict(bind)
    for r, s_ in enumerate(gsym):
        gb[s_] = f"G[{r}]"
    for r, s_ in enumerate(lmsym):
        gb[s_] = f"LM[{r}]"
    lp_j = [(f"lp[{pk(crow[i], lidx(j))}]", sx.mul(gsym[i], jac[i][j])) for i in range(ng) for j in range(nl)
            if not jac[i][j].is_const(0.0)]
    # (J~^T lambda) per stage column, J~ = diag(G) J: the dual-infeasibility and rhs phases
    # read it coalesced instead of gathering NG jacobian entries per variable
    glm = [sx.mul(gsym[r], lmsym[r]) for r in range(ng)]
    jtl_assign = []
    for j in range(nl):
        terms = [sx.mul(glm[r], jac[r][j]) for r in range(ng) if not jac[r][j].is_const(0.0)]
        if terms:
            jtl_assign.append((f"jtl[{j} * S]", sx.sum1(terms)))
    gj_all = g_assign + j_assign + lp_j + jtl_assign

    def emit_gj(net_lds=None):
        lines = sx.CodeGen(gb, prefix="c", net_lds=net_lds).emit(gj_all)
        # the strided jacobian is stored only when requested (scaling, block-chain fallback)
        nj, ntail = len(j_assign), len(lp_j) + len(jtl_assign)
        j_store = lines[len(lines) - ntail - nj:len(lines) - ntail]
        assert all(l.lstrip().startswith("jac[") for l in j_store)
        return (lines[:len(lines) - ntail - nj] + (["  if (full) {"] + j_store + ["  }"] if nj else [])
                + lines[len(lines) - ntail:])

    gj_lines = emit_gj()
    # -- hessian: lower triangle, mirrored; once into the packed local system --
    h_assign = []
    lp_h = []
    for i in range(nl):
        for j in range(i + 1):
            e = hess[i][j]
            if e.is_const(0.0):
                continue
            h_assign.append((f"hess[{i * nl + j} * S]", e))
            if i != j:
                h_assign.append((f"hess[{j * nl + i} * S]", e))
            lp_h.append((f"lp[{pk(lidx(i), lidx(j))}]", e))
    h_all = h_assign + lp_h

    def emit_h(net_lds=None):
        lines = sx.CodeGen(hb, prefix="h", net_lds=net_lds).emit(h_all)
        # the strided full Hessian is stored only when requested (block-chain fallback)
        nh = len(h_assign)
        h_store = lines[len(lines) - nh - len(lp_h):len(lines) - len(lp_h)]
        assert all(l.lstrip().startswith("hess[") for l in h_store)
        return (lines[:len(lines) - nh - len(lp_h)] + (["  if (full) {"] + h_store + ["  }"] if nh else [])
                + lines[len(lines) - len(lp_h):])

    h_lines = emit_h()

    # -- static sparse elimination of the stage interior (runtime/stage_elim.py) --
    P = [[False] * (nloc + 1) for _ in range(nloc + 1)]

    def mark(i, j):
        P[i][j] = P[j][i] = True

    for i in range(nloc + 1):
        P[i][i] = True
    for i in range(nl):
        for j in range(i + 1):
            if not hess[i][j].is_const(0.0):
                mark(lidx(i), lidx(j))
    for r in range(ng):
        for j in range(nl):
            if not jac[r][j].is_const(0.0):
                mark(crow[r], lidx(j))
    for j in range(nloc):  # border (rhs) row: every local index except x_k
        if not (ni <= j < ni + nx):
            mark(nloc, j)
    eq_duals = sorted(crow[r] for r in equality_rows(nlp) if crow[r] < ni) if ng else []
    import math

    pair_w = {}  # preference of a (row, variable) 2x2 pairing: constant entries by magnitude
    for r in range(ng):
        for j in range(nl):
            e = jac[r][j]
            if crow[r] < ni and lidx(j) < nv and not e.is_const(0.0):
                c = e.value if e.is_const() else None
                pair_w[(crow[r], lidx(j))] = (10.0 + max(-5.0, min(5.0, math.log10(abs(c))))) if c else 1.0
    elim_fac, elim_tra, elim_plan = stage_elim.emit(P, ni, nv, nx, nx + nmu, eq_duals, pair_w)
    elim_lines = elim_fac + [stage_elim.CHECK] + elim_tra
    # Stage 0 may open rows that are equalities at k >= 1 (MHE: the link rows of the free
    # x_0 and parameters).  Pairing a variable with such a row makes a 2x2 pivot whose
    # multipliers exceed the growth bound (the row's diagonal is ~1e16 larger than the
    # Jacobian entry), so stage 0 gets a plan of its own with those rows as 1x1 pivots.
    elim0_plan, elim0_lines = None, []
    if ng and nlp.N > 1:
        eq0 = sorted(crow[r] for r in equality_rows(nlp, stage=0) if crow[r] < ni)
        if eq0 != eq_duals:
            f0, t0, elim0_plan = stage_elim.emit(P, ni, nv, nx, nx + nmu, eq0, pair_w)
            elim0_lines = f0 + [stage_elim.CHECK] + t0
    # Equality rows the plan can only pair through a network derivative (NARX output rows)
    # make near-singular 2x2 pivots whenever that entry is small (a saturated sigmoid), and
    # the stage then takes the dense path.  If keeping such rows in the border (their
    # multipliers join the chain, as for bordered continuity rows) leaves an interior whose
    # 2x2 pivots all pair through network-free entries, generate that structure instead.
    if _bordered is None and not nmu and not force_chain and nx > 0:
        col_of = {lidx(j): j for j in range(nl)}

        def network_pairs(plan, lrow_, jac_):
            return sorted(lrow_[d] for b in plan.blocks if len(b) == 2 for v, d in [b]
                          if sx.network_sites([jac_[lrow_[d]][col_of[v]]]))

        weak = network_pairs(elim_plan, lrow, jac)
        if weak and not interior_rank_deficient(nlp, weak):
            alt = generate(nlp, ts, _bordered=weak)
            alt_lrow = [-1] * len(alt.pattern)
            for r, li in enumerate(alt.crow):
                alt_lrow[li] = r
            if not network_pairs(alt.elim, alt_lrow, jac):
                return alt

    # -- compact stage image: structural nonzeros + elimination fill only --
    # order: diagonal (i, i) at i, border row (rhs, j) at nloc + 1 + j, then the other
    # entries of the pattern and of the fill in packed order.  The evaluators write it
    # (lp), the rhs phases its border and the diagonal terms, the kernel copies it to LDS
    # and the generated elimination works on it in place (csrc/mpcx_ipm.hip, factor).
    n_img = nloc + 1
    used_pk = {pk(i, j) for i in range(n_img) for j in range(i + 1) if P[i][j]}
    for ln in elim_lines + elim0_lines:
        used_pk.update(int(m.group(1)) for m in re.finditer(r"F\[(\d+)\]", ln))
    unpk = {pk(i, j): (i, j) for i in range(n_img) for j in range(i + 1)}
    compact = [(i, i) for i in range(n_img)] + [(nloc, j) for j in range(nloc)]
    head = {pk(i, j) for i, j in compact}
    compact += [unpk[t] for t in sorted(used_pk - head)]
    cix = {pk(i, j): c for c, (i, j) in enumerate(compact)}

    def to_compact(lines, arr):
        # lp (the evaluators' image in HBM) is stage-minor: entry c of the stage at lp[c * S]
        stride = " * S" if arr == "lp" else ""
        return [re.sub(rf"\b{arr}\[(\d+)\]", lambda m: f"{arr}[{cix[int(m.group(1))]}{stride}]", ln)
                for ln in lines]

    elim_lines = to_compact(elim_lines, "F")
    elim0_lines = to_compact(elim0_lines, "F")
    gj_lines = to_compact(gj_lines, "lp")
    h_lines = to_compact(h_lines, "lp")

    net_lines, net_defs, netx, neto = _network_section(nlp, bind, fg_assign, gj_all, h_all, emit_gj, emit_h,
                                                       to_compact)

    dims = dict(N=nlp.N, NX=nlp.nx, NV=nlp.nv, NG=ng, NPS=nlp.nps, NPG=nlp.npg)
    ts = nlp.ts if ts is None else ts
    flops = {
        "fg": sx.flop_count([st.cost] + list(st.g)),
        "gj": sx.flop_count([e for _, e in gj_assign]),
        "hess": sx.flop_count([e for _, e in h_assign]),
    }
    nnz = {"jac": sum(1 for a, _ in gj_assign if a.startswith("jac")),
           "hess": sum(1 for a, _ in h_assign)}

    sig = "const double* __restrict__ L, const double* __restrict__ PS, const double* __restrict__ PG, const double TK"
    out: List[str] = [
        "// generated by agentlib_mpc_amd.runtime.codegen — do not edit",
        f"#define MPCX_N {nlp.N}",
        f"#define MPCX_NX {nlp.nx}",
        f"#define MPCX_NV {nlp.nv}",
        f"#define MPCX_NG {ng}",
        f"#define MPCX_NPS {nlp.nps}",
        f"#define MPCX_NPG {nlp.npg}",
        f"#define MPCX_TS {float(ts)!r}",
        f"#define MPCX_ABI {KERNEL_ABI_VERSION}",
        f"#define MPCX_NCPT {len(compact)}",
        f"#define MPCX_CPK_INIT {', '.join(str(pk(i, j)) for i, j in compact)}",
        f"#define MPCX_CIJ_INIT {', '.join(str(i | (j << 8)) for i, j in compact)}",
        *(["#define MPCX_FORCE_BLOCK_CHAIN 1"] if force_chain else []),
        *([f"#define MPCX_NMU {nmu}",
           f"#define MPCX_CROW_INIT {', '.join(map(str, crow))}",
           f"#define MPCX_LROW_INIT {', '.join(map(str, lrow))}"] if nmu else []),
        "#include <hip/hip_runtime.h>",
        "#include <math.h>",
        "",
        f"__device__ __forceinline__ void gen_stage_fg({sig}, double* __restrict__ f, double* __restrict__ g, const int S) {{",
        *fg_lines, "}", "",
        "__device__ __forceinline__ void gen_stage_bounds(const double* __restrict__ PS, const double* __restrict__ PG, const double TK, double* __restrict__ lb, double* __restrict__ ub, const int S) {",
        *bd_lines, "}", "",
        f"__device__ __forceinline__ void gen_stage_gj({sig}, double* __restrict__ grad, double* __restrict__ jac, const int S, const double* __restrict__ G, double* __restrict__ lp, const double* __restrict__ LM, double* __restrict__ jtl, const int full) {{",
        *gj_lines, "}", "",
        f"__device__ __forceinline__ void gen_stage_hess({sig}, const double sigma, const double* __restrict__ lam, double* __restrict__ hess, const int S, double* __restrict__ lp, const int full) {{",
        *h_lines, "}", "",
        "// >>> device only: static sparse elimination of the stage interior (runtime/stage_elim.py):",
        f"// {len(elim_plan.blocks)} pivot blocks, {elim_plan.n_update} interior updates, {elim_plan.nnz_l} multipliers",
        "#define MPCX_STATIC_ELIM 1",
        "#ifndef MPCX_ELIM_GROWTH  // threshold-pivoting bound on the static multipliers (runtime/stage_elim.py)",
        "#define MPCX_ELIM_GROWTH 1e8",
        "#endif",
        "// reciprocals of pivots and slacks (mpcx_ipm.hip): v_rcp_f64 (2^-23 relative) refined by two",
        "// Newton steps to within an ulp -- five dependent instructions instead of the eleven of an",
        "// IEEE division (scaling, fixup); MPCX_IEEE_DIV keeps the division (A/B builds)",
        "#ifndef MPCX_RCP",
        "#ifdef MPCX_IEEE_DIV",
        "__device__ __forceinline__ double mpcx_frcp(double x) { return 1.0 / x; }",
        "#else",
        "__device__ __forceinline__ double mpcx_frcp(double x) {",
        "  const double r0 = __builtin_amdgcn_rcp(x);",
        "  double r = fma(fma(-x, r0, 1.0), r0, r0);",
        "  r = fma(fma(-x, r, 1.0), r, r);",
        "  // 0, +-inf, NaN (x = +-inf, +-0, NaN or overflowing): v_rcp_f64's IEEE value, which the",
        "  // Newton steps would turn into NaN (-0 * inf)",
        "  return __builtin_amdgcn_class(r0, 0x267) ? r0 : r;  // classes snan | qnan | -inf | -0 | +0 | +inf",
        "}",
        "#endif",
        "#define MPCX_RCP(x) mpcx_frcp(x)",
        "#endif",
        "#ifndef MPCX_ELIM_FENCE  // scheduling fence between pivot blocks (register pressure)",
        "#define MPCX_ELIM_FENCE __builtin_amdgcn_sched_barrier(0)",
        "#endif",
        "typedef __attribute__((address_space(3))) double mpcx_elim_ld;",
        "// F: the stage image the elimination works on -- LDS, or a register array the eliminating lane\n"
        "// loads it into (mpcx_ipm.hip static_stage, ELIM_REG)",
        "#ifdef MPCX_WS_LDS  // small-fleet build: the workspace (operators, pivot order) is in LDS",
        "typedef __attribute__((address_space(3))) double mpcx_elim_gd;",
        "typedef __attribute__((address_space(3))) int mpcx_elim_gi;",
        "#else",
        "typedef __attribute__((address_space(1))) double mpcx_elim_gd;",
        "typedef __attribute__((address_space(1))) int mpcx_elim_gi;",
        "#endif",
        "template <typename FD> __device__ __forceinline__ int gen_stage_elim(FD* __restrict__ F, mpcx_elim_ld* __restrict__ S, mpcx_elim_ld* __restrict__ ZX, mpcx_elim_gd* __restrict__ TR, mpcx_elim_gi* __restrict__ PRM, int* __restrict__ inert) {",
        "  int bad = 0, pos = 0, neg = 0;",
        *elim_lines,
        "  inert[0] = pos; inert[1] = neg; inert[2] = 0;",
        "  return 0;",
        "}",
        *([f"// stage 0: {len(elim0_plan.blocks)} pivot blocks, {elim0_plan.n_update} interior updates "
           f"(rows open at k = 0 are 1x1 pivots)",
           "#define MPCX_STATIC_ELIM0 1",
           "template <typename FD> __device__ __forceinline__ int gen_stage_elim0(FD* __restrict__ F, mpcx_elim_ld* __restrict__ S, mpcx_elim_ld* __restrict__ ZX, mpcx_elim_gd* __restrict__ TR, mpcx_elim_gi* __restrict__ PRM, int* __restrict__ inert) {",
           "  int bad = 0, pos = 0, neg = 0;",
           *elim0_lines,
           "  inert[0] = pos; inert[1] = neg; inert[2] = 0;",
           "  return 0;",
           "}"] if elim0_plan is not None else []),
        *net_defs,
        *net_lines,
        "// <<< device only", "",
        '#include "mpcx_ipm.hip"',
        "",
    ]
    src = "\n".join(out)
    # network weight tables; ids renumbered by first use so the source is deterministic
    used = []
    for m in re.finditer(r"ANN(\d+)_", src):
        if int(m.group(1)) not in used:
            used.append(int(m.group(1)))
    if used:
        local = {nid: i for i, nid in enumerate(used)}
        tables = sx.network_tables(used)
        src = src.replace('#include <math.h>\n', '#include <math.h>\n' + "\n".join(tables) + "\n", 1)
        src = re.sub(r"ANN(\d+)_", lambda m: f"ANN{local[int(m.group(1))]}_", src)
    key = hashlib.sha1(src.encode()).hexdigest()[:16]
    return GeneratedModel(source=src, key=key, dims=dims, flops=flops, nnz=nnz, block_chain_only=force_chain,
                          bordered_rows=list(bordered), elim=elim_plan, elim_lines=elim_lines, pattern=P,
                          compact=compact, crow=crow, elim0=elim0_plan, elim0_lines=elim0_lines)
