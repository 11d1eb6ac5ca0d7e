"""Scalar symbolic expressions: the tracer, AD and code generator of this backend.

The reference builds its NLPs with CasADi ``MX``/``SX`` symbols and lets
``nlpsol(..., {"expand": True})`` turn them into straight-line scalar graphs
(`agentlib_mpc/data_structures/casadi_utils.py:191-217`).  CasADi is not part of
this framework; models written against the ``CasadiModel`` API
(`agentlib_mpc/models/casadi_model.py:36-152`) are traced into the hash-consed
DAG below instead.  It supports the operator subset the reference models use
(``+ - * / **``, unary minus, ``exp log sqrt tanh sin cos fabs fmax fmin
if_else`` and comparisons), symbolic forward differentiation (for gradients,
Jacobians and Lagrangian Hessians) and emission of straight-line C/HIP code.

Nodes are interned: building the same (op, args) twice returns the same object,
so common sub-expressions are shared automatically and code generation emits
each node once.
"""

from __future__ import annotations

import math
import numbers
from typing import Dict, Iterable, List, Sequence, Tuple, Union

import numpy as np

__all__ = [
    "Expr", "SX", "sym", "const", "as_expr", "exp", "log", "sqrt", "tanh", "sin",
    "cos", "fabs", "fmax", "fmin", "if_else", "sum1", "diff", "gradient",
    "jacobian", "hessian", "substitute", "free_symbols", "evaluate", "CodeGen",
    "inf",
]

inf = math.inf

_UNARY = {"neg", "exp", "log", "sqrt", "tanh", "sin", "cos", "fabs", "sq"}
_BINARY = {"add", "sub", "mul", "div", "pow", "fmax", "fmin", "lt", "le", "eq", "ne"}


class Expr:
    """A node of the scalar expression DAG (interned)."""

    __slots__ = ("op", "args", "value", "name", "uid", "__weakref__")
    _table: Dict[tuple, "Expr"] = {}
    _counter = 0

    def __new__(cls, op: str, args: tuple = (), value=None, name: str = None):
        if op == "sym":
            key = None  # symbols are never merged
        elif op == "const":
            v = float(value)
            # -0.0 and 0.0 compare equal; keep one representative
            key = ("const", 0.0 if v == 0.0 else v) if not math.isnan(v) else None
        else:
            key = (op, tuple(a.uid for a in args))
        if key is not None:
            hit = cls._table.get(key)
            if hit is not None:
                return hit
        obj = object.__new__(cls)
        obj.op = op
        obj.args = args
        obj.value = None if value is None else float(value)
        obj.name = name
        Expr._counter += 1
        obj.uid = Expr._counter
        if key is not None:
            cls._table[key] = obj
        return obj

    # -- python protocol -------------------------------------------------------
    def __repr__(self):
        return to_string(self)

    def __hash__(self):
        return self.uid

    # nodes are immutable and interned: copies are the node itself
    def __copy__(self):
        return self

    def __deepcopy__(self, memo):
        return self

    def is_const(self, v=None) -> bool:
        return self.op == "const" and (v is None or self.value == v)

    @property
    def shape(self):
        return (1, 1)

    def __float__(self):
        if self.op == "const":
            return self.value
        raise TypeError(f"Cannot convert non-constant expression {self} to float")

    # arithmetic
    def __add__(self, o):
        return add(self, o)

    def __radd__(self, o):
        return add(o, self)

    def __sub__(self, o):
        return sub(self, o)

    def __rsub__(self, o):
        return sub(o, self)

    def __mul__(self, o):
        return mul(self, o)

    def __rmul__(self, o):
        return mul(o, self)

    def __truediv__(self, o):
        return div(self, o)

    def __rtruediv__(self, o):
        return div(o, self)

    def __pow__(self, o, modulo=None):
        return power(self, o)

    def __rpow__(self, o):
        return power(o, self)

    def __neg__(self):
        return neg(self)

    def __pos__(self):
        return self

    def __abs__(self):
        return fabs(self)

    # comparisons build expressions (as CasADi does); equality of python
    # objects is identity because nodes are interned
    def __lt__(self, o):
        return _cmp("lt", self, o)

    def __le__(self, o):
        return _cmp("le", self, o)

    def __gt__(self, o):
        return _cmp("lt", o, self)

    def __ge__(self, o):
        return _cmp("le", o, self)

    def __eq__(self, o):  # noqa: D105 - identity semantics kept for dict keys
        if isinstance(o, Expr):
            return self is o
        return NotImplemented

    __array_priority__ = 1000


SX = Expr


def const(v: float) -> Expr:
    return Expr("const", value=v)


ZERO = const(0.0)
ONE = const(1.0)


def sym(name: str) -> Expr:
    return Expr("sym", name=name)


def as_expr(x) -> Expr:
    if isinstance(x, Expr):
        return x
    if hasattr(x, "sym") and isinstance(getattr(x, "sym"), Expr):
        return x.sym
    if isinstance(x, (numbers.Real, np.floating, np.integer, bool)):
        return const(float(x))
    if isinstance(x, np.ndarray) and x.size == 1:
        return const(float(x.reshape(-1)[0]))
    raise TypeError(f"Cannot convert {type(x)} to a symbolic expression")


def _binary(op, a, b):
    return Expr(op, (a, b))


def add(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(a.value + b.value)
    if a.is_const(0.0):
        return b
    if b.is_const(0.0):
        return a
    if b.op == "neg":
        return sub(a, b.args[0])
    return _binary("add", a, b)


def sub(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(a.value - b.value)
    if b.is_const(0.0):
        return a
    if a.is_const(0.0):
        return neg(b)
    if a is b:
        return ZERO
    if b.op == "neg":
        return add(a, b.args[0])
    return _binary("sub", a, b)


def mul(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(a.value * b.value)
    # CasADi's SX simplifier also drops multiplications by structural zeros
    if a.is_const(0.0) or b.is_const(0.0):
        return ZERO
    if a.is_const(1.0):
        return b
    if b.is_const(1.0):
        return a
    if a.is_const(-1.0):
        return neg(b)
    if b.is_const(-1.0):
        return neg(a)
    if a is b:
        return Expr("sq", (a,))
    return _binary("mul", a, b)


def div(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(a.value / b.value) if b.value != 0 else const(math.copysign(math.inf, a.value) if a.value else math.nan)
    if a.is_const(0.0):
        return ZERO
    if b.is_const(1.0):
        return a
    if b.is_const(-1.0):
        return neg(a)
    return _binary("div", a, b)


def neg(a) -> Expr:
    a = as_expr(a)
    if a.op == "const":
        return const(-a.value)
    if a.op == "neg":
        return a.args[0]
    return Expr("neg", (a,))


def power(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(a.value ** b.value)
    if b.op == "const":
        if b.value == 0.0:
            return ONE
        if b.value == 1.0:
            return a
        if b.value == 2.0:
            return Expr("sq", (a,))
        if b.value == -1.0:
            return div(ONE, a)
        if b.value == 0.5:
            return sqrt(a)
    return _binary("pow", a, b)


def _unary_fold(op, fn):
    def f(a) -> Expr:
        a = as_expr(a)
        if a.op == "const":
            return const(fn(a.value))
        return Expr(op, (a,))

    f.__name__ = op
    return f


def _safe(fn):
    def g(v):
        try:
            return fn(v)
        except (ValueError, OverflowError):
            return math.nan

    return g


exp = _unary_fold("exp", _safe(math.exp))
log = _unary_fold("log", _safe(lambda v: math.log(v) if v > 0 else (-math.inf if v == 0 else math.nan)))
sqrt = _unary_fold("sqrt", _safe(math.sqrt))
tanh = _unary_fold("tanh", math.tanh)
sin = _unary_fold("sin", math.sin)
cos = _unary_fold("cos", math.cos)
fabs = _unary_fold("fabs", abs)


def sq(a) -> Expr:
    a = as_expr(a)
    if a.op == "const":
        return const(a.value * a.value)
    return Expr("sq", (a,))


def fmax(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(max(a.value, b.value))
    return _binary("fmax", a, b)


def fmin(a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        return const(min(a.value, b.value))
    return _binary("fmin", a, b)


def _cmp(op, a, b) -> Expr:
    a, b = as_expr(a), as_expr(b)
    if a.op == "const" and b.op == "const":
        fn = {"lt": a.value < b.value, "le": a.value <= b.value,
              "eq": a.value == b.value, "ne": a.value != b.value}[op]
        return const(1.0 if fn else 0.0)
    return _binary(op, a, b)


def if_else(cond, a, b, short_circuit: bool = False) -> Expr:
    """``cond ? a : b`` with the CasADi argument order (`ca.if_else`)."""
    cond, a, b = as_expr(cond), as_expr(a), as_expr(b)
    if cond.op == "const":
        return a if cond.value != 0 else b
    if a is b:
        return a
    return Expr("if_else", (cond, a, b))


def sum1(items: Iterable) -> Expr:
    out = ZERO
    for it in items:
        out = add(out, it)
    return out


# ---------------------------------------------------------------------------
# opaque one-hidden-layer networks (the NARX models of the ML backends)
# ---------------------------------------------------------------------------
#
# A network y = b2 + sum_j w2_j act(b1_j + sum_i W1_ij x_i) is one n-ary node
# ``annv<id>`` instead of its expanded graph.  Its derivatives are nodes too:
# ``annd<id>_<i>`` = dy/dx_i and ``anndd<id>_<i>_<k>`` (i >= k) = d2y/dx_i dx_k,
# so gradients and Lagrangian Hessians stay compact, and the code generator
# evaluates each network once per stage in a loop over the hidden units with
# the weights in constant memory (only the derivative entries that are used).

_ACTS = ("sigmoid", "tanh", "linear", "softplus", "exponential", "gaussian")


class Network:
    """Dense weights of a single-hidden-layer, single-output network."""

    def __init__(self, W1: np.ndarray, b1: np.ndarray, w2: np.ndarray, b2: float, act: str):
        if act not in _ACTS:
            raise ValueError(f"activation {act!r} has no smooth closed-form derivatives")
        self.W1 = np.ascontiguousarray(W1, dtype=float)   # [n_in, H]
        self.b1 = np.asarray(b1, dtype=float).reshape(-1)
        self.w2 = np.asarray(w2, dtype=float).reshape(-1)
        self.b2 = float(b2)
        self.act = act
        self.n_in, self.H = self.W1.shape

    def key(self) -> tuple:
        return (self.act, self.b2, self.W1.tobytes(), self.b1.tobytes(), self.w2.tobytes())

    def act_derivs(self, a):
        """act(a), act'(a), act''(a) (numpy)."""
        if self.act == "sigmoid":
            s = 1.0 / (1.0 + np.exp(-a))
            s1 = s * (1.0 - s)
            return s, s1, s1 * (1.0 - 2.0 * s)
        if self.act == "tanh":
            t = np.tanh(a)
            t1 = 1.0 - t * t
            return t, t1, -2.0 * t * t1
        if self.act == "linear":
            return a, np.ones_like(a), np.zeros_like(a)
        if self.act == "softplus":
            s = 1.0 / (1.0 + np.exp(-a))
            return np.log(1.0 + np.exp(a)), s, s * (1.0 - s)
        if self.act == "exponential":
            e = np.exp(a)
            return e, e, e
        g = np.exp(-a * a)  # gaussian
        return g, -2.0 * a * g, (4.0 * a * a - 2.0) * g

    def evaluate(self, x: np.ndarray):
        """value [...], gradient [..., n_in], Hessian [..., n_in, n_in] on rows x [..., n_in]."""
        a = x @ self.W1 + self.b1
        s0, s1, s2 = self.act_derivs(a)
        v = s0 @ self.w2 + self.b2
        g = (s1 * self.w2) @ self.W1.T
        h = np.einsum("...j,ij,kj->...ik", s2 * self.w2, self.W1, self.W1)
        return v, g, h


_NETWORKS: List[Network] = []
_NETWORK_IDS: Dict[tuple, int] = {}


def register_network(net: Network) -> int:
    """Intern a network; identical weights share one id."""
    k = net.key()
    if k not in _NETWORK_IDS:
        _NETWORK_IDS[k] = len(_NETWORKS)
        _NETWORKS.append(net)
    return _NETWORK_IDS[k]


def network(net_id: int) -> Network:
    return _NETWORKS[net_id]


def ann_call(net_id: int, inputs: Sequence) -> Expr:
    """Output of network ``net_id`` at ``inputs`` (one node)."""
    args = tuple(as_expr(x) for x in inputs)
    if len(args) != _NETWORKS[net_id].n_in:
        raise ValueError("network input size mismatch")
    return Expr(f"annv{net_id}", args)


def ann_parse(op: str):
    """(kind, net id, i, k) of a network op, or None: kind in {'v', 'd', 'dd'}."""
    if not op.startswith("ann"):
        return None
    if op.startswith("annv"):
        return "v", int(op[4:]), -1, -1
    if op.startswith("anndd"):
        nid, i, k = op[5:].split("_")
        return "dd", int(nid), int(i), int(k)
    nid, i = op[4:].split("_")
    return "d", int(nid), int(i), -1


def _ann_node(kind: str, nid: int, args, i: int = -1, k: int = -1) -> Expr:
    if kind == "d":
        return Expr(f"annd{nid}_{i}", tuple(args))
    i, k = max(i, k), min(i, k)
    return Expr(f"anndd{nid}_{i}_{k}", tuple(args))


# ---------------------------------------------------------------------------
# traversal helpers
# ---------------------------------------------------------------------------

def topo_order(outputs: Sequence[Expr]) -> List[Expr]:
    """Post-order (children first) list of all nodes reachable from outputs."""
    seen = set()
    order: List[Expr] = []
    for root in outputs:
        root = as_expr(root)
        if root.uid in seen:
            continue
        stack = [(root, False)]
        while stack:
            node, expanded = stack.pop()
            if expanded:
                order.append(node)
                continue
            if node.uid in seen:
                continue
            seen.add(node.uid)
            stack.append((node, True))
            for a in reversed(node.args):
                if a.uid not in seen:
                    stack.append((a, False))
    return order


def free_symbols(outputs: Sequence[Expr]) -> List[Expr]:
    return [n for n in topo_order(outputs) if n.op == "sym"]


def depends_on(e: Expr, syms: Iterable[Expr]) -> bool:
    ids = {s.uid for s in syms}
    return any(n.uid in ids for n in topo_order([e]))


def substitute(outputs: Sequence[Expr], mapping: Dict[Expr, Union[Expr, float]]) -> List[Expr]:
    """Replace symbols (or any node) by other expressions, rebuilding the DAG."""
    repl = {k.uid: as_expr(v) for k, v in mapping.items()}
    memo: Dict[int, Expr] = {}
    outs = [as_expr(o) for o in outputs]
    for node in topo_order(outs):
        if node.uid in repl:
            memo[node.uid] = repl[node.uid]
            continue
        if node.op in ("sym", "const"):
            memo[node.uid] = node
            continue
        new_args = [memo[a.uid] for a in node.args]
        memo[node.uid] = _rebuild(node.op, new_args)
    return [memo[o.uid] for o in outs]


def strip_squares(e) -> Tuple[Expr, bool]:
    """``e`` with every ``sq(a)`` node replaced by ``a``, and whether there was one: the
    reference's stats evaluator turns the printed ``sq(`` into ``(`` and squares the
    whole term instead (`data_structures/objective.py:166-224`)."""
    e = as_expr(e)
    memo: Dict[int, Expr] = {}
    found = False
    for node in topo_order([e]):
        if node.op in ("sym", "const"):
            memo[node.uid] = node
        elif node.op == "sq":
            memo[node.uid] = memo[node.args[0].uid]
            found = True
        else:
            memo[node.uid] = _rebuild(node.op, [memo[a.uid] for a in node.args])
    return memo[e.uid], found


def _rebuild(op: str, args: List[Expr]) -> Expr:
    if op.startswith("ann"):
        return Expr(op, tuple(args))
    if op == "add":
        return add(*args)
    if op == "sub":
        return sub(*args)
    if op == "mul":
        return mul(*args)
    if op == "div":
        return div(*args)
    if op == "neg":
        return neg(args[0])
    if op == "pow":
        return power(*args)
    if op == "sq":
        return sq(args[0])
    if op in ("lt", "le", "eq", "ne"):
        return _cmp(op, *args)
    if op == "fmax":
        return fmax(*args)
    if op == "fmin":
        return fmin(*args)
    if op == "if_else":
        return if_else(*args)
    return {"exp": exp, "log": log, "sqrt": sqrt, "tanh": tanh, "sin": sin,
            "cos": cos, "fabs": fabs}[op](args[0])


# ---------------------------------------------------------------------------
# differentiation
# ---------------------------------------------------------------------------

def diff(e, x: Expr, _memo: Dict[int, Expr] = None) -> Expr:
    """Symbolic derivative d e / d x (x must be a symbol)."""
    e = as_expr(e)
    if _memo is None:
        _memo = {}
    for node in topo_order([e]):
        if node.uid in _memo:
            continue
        _memo[node.uid] = _diff_node(node, x, _memo)
    return _memo[e.uid]


def _diff_node(n: Expr, x: Expr, m: Dict[int, Expr]) -> Expr:
    op = n.op
    if op == "sym":
        return ONE if n is x else ZERO
    if op == "const":
        return ZERO
    if op.startswith("ann"):
        kind, nid, i, _ = ann_parse(op)
        if kind == "dd":
            raise NotImplementedError("third derivatives of networks are not needed by the solver")
        out = ZERO
        for j, a in enumerate(n.args):
            da = m[a.uid]
            if da.is_const(0.0):
                continue
            dn = _ann_node("d", nid, n.args, j) if kind == "v" else _ann_node("dd", nid, n.args, i, j)
            out = add(out, mul(dn, da))
        return out
    a = n.args[0]
    da = m[a.uid]
    if op == "neg":
        return neg(da)
    if op == "add":
        return add(da, m[n.args[1].uid])
    if op == "sub":
        return sub(da, m[n.args[1].uid])
    if op == "mul":
        b = n.args[1]
        db = m[b.uid]
        return add(mul(da, b), mul(a, db))
    if op == "div":
        b = n.args[1]
        db = m[b.uid]
        # (da*b - a*db)/b^2 == da/b - (a/b)*db/b
        t1 = div(da, b)
        t2 = mul(div(n, b), db) if not db.is_const(0.0) else ZERO
        return sub(t1, t2)
    if op == "sq":
        return mul(mul(const(2.0), a), da)
    if op == "pow":
        b = n.args[1]
        db = m[b.uid]
        if b.op == "const":
            return mul(mul(b, power(a, const(b.value - 1.0))), da)
        # d(a^b) = a^b (db log a + b da / a)
        return mul(n, add(mul(db, log(a)), div(mul(b, da), a)))
    if op == "exp":
        return mul(n, da)
    if op == "log":
        return div(da, a)
    if op == "sqrt":
        return div(da, mul(const(2.0), n))
    if op == "tanh":
        return mul(sub(ONE, sq(n)), da)
    if op == "sin":
        return mul(cos(a), da)
    if op == "cos":
        return neg(mul(sin(a), da))
    if op == "fabs":
        # sign(a) * da, sign as if_else to keep it straight-line
        return mul(if_else(_cmp("lt", a, ZERO), const(-1.0), ONE), da)
    if op in ("fmax", "fmin"):
        b = n.args[1]
        db = m[b.uid]
        cond = _cmp("le", b, a) if op == "fmax" else _cmp("le", a, b)
        return if_else(cond, da, db)
    if op == "if_else":
        c, t, f = n.args
        return if_else(c, m[t.uid], m[f.uid])
    if op in ("lt", "le", "eq", "ne"):
        return ZERO
    raise NotImplementedError(op)


def gradient(f, xs: Sequence[Expr]) -> List[Expr]:
    f = as_expr(f)
    return [diff(f, x) for x in xs]


def jacobian(fs: Sequence, xs: Sequence[Expr]) -> List[List[Expr]]:
    return [[diff(as_expr(f), x) for x in xs] for f in fs]


def hessian(f, xs: Sequence[Expr]) -> List[List[Expr]]:
    g = gradient(f, xs)
    return [[diff(gi, xj) for xj in xs] for gi in g]


# ---------------------------------------------------------------------------
# numeric evaluation (vectorised over a leading batch axis)
# ---------------------------------------------------------------------------

def evaluate(outputs: Sequence, values: Dict[Expr, Union[float, np.ndarray]]) -> List[np.ndarray]:
    """Evaluate expressions with numpy; values may be arrays (broadcast)."""
    outs = [as_expr(o) for o in outputs]
    vals: Dict[int, object] = {}
    for k, v in values.items():
        vals[as_expr(k).uid] = np.asarray(v, dtype=float)
    with np.errstate(all="ignore"):
        for n in topo_order(outs):
            if n.uid in vals:
                continue
            op = n.op
            if op == "const":
                vals[n.uid] = np.float64(n.value)
                continue
            if op == "sym":
                raise KeyError(f"No value for symbol {n.name}")
            a = [vals[x.uid] for x in n.args]
            if op.startswith("ann"):
                kind, nid, i, k = ann_parse(op)
                xs = np.stack(np.broadcast_arrays(*a), axis=-1)
                v, g, h = _NETWORKS[nid].evaluate(xs)
                vals[n.uid] = v if kind == "v" else (g[..., i] if kind == "d" else h[..., i, k])
                continue
            vals[n.uid] = _NUMPY_OPS[op](*a)
    return [np.asarray(vals[o.uid], dtype=float) for o in outs]


_NUMPY_OPS = {
    "add": np.add, "sub": np.subtract, "mul": np.multiply, "div": np.divide,
    "neg": np.negative, "pow": np.power, "sq": np.square, "exp": np.exp,
    "log": np.log, "sqrt": np.sqrt, "tanh": np.tanh, "sin": np.sin, "cos": np.cos,
    "fabs": np.abs, "fmax": np.fmax, "fmin": np.fmin,
    "lt": lambda a, b: (a < b).astype(float), "le": lambda a, b: (a <= b).astype(float),
    "eq": lambda a, b: (a == b).astype(float), "ne": lambda a, b: (a != b).astype(float),
    "if_else": lambda c, t, f: np.where(c != 0, t, f),
}


def to_string(e: Expr, _depth: int = 0) -> str:
    if e.op == "const":
        return repr(e.value)
    if e.op == "sym":
        return e.name
    if _depth > 12:
        return "..."
    a = [to_string(x, _depth + 1) for x in e.args]
    infix = {"add": "+", "sub": "-", "mul": "*", "div": "/", "lt": "<", "le": "<=",
             "eq": "==", "ne": "!="}
    if e.op in infix:
        return f"({a[0]}{infix[e.op]}{a[1]})"
    if e.op == "neg":
        return f"(-{a[0]})"
    if e.op == "pow":
        return f"pow({a[0]},{a[1]})"
    return f"{e.op}({', '.join(a)})"


def count_ops(outputs: Sequence[Expr]) -> Dict[str, int]:
    """Floating point operation count of the DAG (shared nodes counted once)."""
    counts: Dict[str, int] = {}
    for n in topo_order([as_expr(o) for o in outputs]):
        if n.op in ("sym", "const"):
            continue
        counts[n.op] = counts.get(n.op, 0) + 1
    return counts


def flop_count(outputs: Sequence[Expr]) -> int:
    nodes = topo_order([as_expr(o) for o in outputs])
    groups: Dict[tuple, set] = {}
    for n in nodes:
        pa = ann_parse(n.op) if n.op.startswith("ann") else None
        if pa is not None:
            groups.setdefault((pa[1], tuple(a.uid for a in n.args)), set()).add(pa[0] + str(pa[2]) + str(pa[3]))
    ann_flops = 0
    for (nid, _), used in groups.items():
        net = _NETWORKS[nid]
        # pre-activation + activation (+ derivatives) + one FMA per used output entry
        ann_flops += net.H * (2 * net.n_in + 14 + 2 * len(used))
    c = {k: v for k, v in count_ops(outputs).items() if not k.startswith("ann")}
    # transcendental functions are priced as a handful of flops
    weights = {"exp": 8, "log": 8, "sqrt": 4, "tanh": 10, "sin": 8, "cos": 8,
               "pow": 16, "div": 4}
    return int(sum(v * weights.get(k, 1) for k, v in c.items())) + ann_flops


# ---------------------------------------------------------------------------
# code generation
# ---------------------------------------------------------------------------

def _c_literal(v: float) -> str:
    if math.isnan(v):
        return "__builtin_nan(\"\")"
    if math.isinf(v):
        return "(__builtin_inf())" if v > 0 else "(-__builtin_inf())"
    r = repr(float(v))
    if "e" not in r and "." not in r and "inf" not in r:
        r += ".0"
    return r


class CodeGen:
    """Emit straight-line C for a set of outputs.

    ``inputs`` maps symbols to C l-value expressions; ``emit`` returns the body
    lines assigning each output expression to the given C target.  Network
    nodes (``annv/annd/anndd``) sharing one input tuple are evaluated together
    by one loop over the hidden units (weights ``ANN<id>_*`` in constant memory,
    see :func:`network_tables`); ``networks`` collects the ids used.
    """

    def __init__(self, inputs: Dict[Expr, str], prefix: str = "t", net_lds=None):
        self.inputs = {k.uid: v for k, v in inputs.items()}
        self.prefix = prefix
        self.networks = set()
        #: optional ``(nid, arg uids, member key) -> C expression``: network entries are read
        #: from values a wave-level pass computed (MFMA, csrc/mpcx_net_mfma.h) instead of
        #: being evaluated by the hidden-unit loop
        self.net_lds = net_lds

    def emit(self, assignments: Sequence[Tuple[str, Expr]], indent: str = "  ") -> List[str]:
        outs = [as_expr(e) for _, e in assignments]
        order = topo_order(outs)
        groups: Dict[tuple, Dict[tuple, Expr]] = {}
        for n in order:
            pa = ann_parse(n.op) if n.op.startswith("ann") else None
            if pa is not None:
                groups.setdefault((pa[1], tuple(a.uid for a in n.args)), {})[pa[0], pa[2], pa[3]] = n
        names: Dict[int, str] = {}
        lines: List[str] = []
        n_groups = 0
        # denominators divided by more than once: ONE reciprocal, then products (r05: the MHE
        # Hessian divided by the same capacity term ten times per stage; a division is eleven
        # dependent instructions on the GPU).  The products agree with the quotients to an ulp.
        # (constant denominators keep their divisions: x / 10.0 is not x * 0.1)
        den_uses: Dict[int, int] = {}
        for n in order:
            if n.op == "div" and n.args[1].op != "const":
                den_uses[n.args[1].uid] = den_uses.get(n.args[1].uid, 0) + 1
        recips: Dict[int, str] = {}
        for n in order:
            if n.uid in names:
                continue
            if n.op == "const":
                names[n.uid] = _c_literal(n.value)
                continue
            if n.op == "sym":
                if n.uid not in self.inputs:
                    raise KeyError(f"Symbol {n.name} has no input binding in code generation")
                names[n.uid] = self.inputs[n.uid]
                continue
            a = [names[x.uid] for x in n.args]
            if n.op.startswith("ann"):
                nid = ann_parse(n.op)[1]
                members = groups[(nid, tuple(x.uid for x in n.args))]
                gp = f"{self.prefix}n{n_groups}"
                n_groups += 1
                if self.net_lds is not None:
                    key = tuple(x.uid for x in n.args)
                    for mk, node in members.items():
                        var = f"{gp}{'v' if mk[0] == 'v' else ('g%d' % mk[1] if mk[0] == 'd' else 'h%d_%d' % mk[1:])}"
                        lines.append(f"{indent}const double {var} = {self.net_lds(nid, key, mk)};")
                        names[node.uid] = var
                    self.networks.add(nid)
                    continue
                lines += _emit_network(nid, a, members, gp, names, indent)
                self.networks.add(nid)
                continue
            if n.op == "div" and den_uses.get(n.args[1].uid, 0) > 1:
                du = n.args[1].uid
                if du not in recips:
                    recips[du] = f"{self.prefix}{len(lines)}"
                    lines.append(f"{indent}const double {recips[du]} = 1.0 / {a[1]};")
                expr = f"{a[0]} * {recips[du]}"
            else:
                expr = _c_op(n.op, a)
            # temporaries are numbered in emission order (not by node uid), so the
            # generated source -- and the code-object cache key -- is independent of
            # what else the process has traced before
            var = f"{self.prefix}{len(lines)}"
            lines.append(f"{indent}const double {var} = {expr};")
            names[n.uid] = var
        for target, e in assignments:
            lines.append(f"{indent}{target} = {names[as_expr(e).uid]};")
        return lines


def network_sites(outputs: Sequence[Expr]) -> Dict[tuple, Tuple[int, tuple, Dict[tuple, Expr]]]:
    """Network call sites of a DAG in topological order: ``(nid, arg uids) -> (nid, args,
    {member key: node})`` with member keys ``('v', -1, -1)``, ``('d', i, -1)``, ``('dd', i, k)``."""
    sites: Dict[tuple, Tuple[int, tuple, Dict[tuple, Expr]]] = {}
    for n in topo_order([as_expr(o) for o in outputs]):
        pa = ann_parse(n.op) if n.op.startswith("ann") else None
        if pa is None:
            continue
        key = (pa[1], tuple(a.uid for a in n.args))
        sites.setdefault(key, (pa[1], n.args, {}))[2][pa[0], pa[2], pa[3]] = n
    return sites


#: activation codes of the wave-level network pass (csrc/mpcx_net_mfma.h)
ACT_CODE = {a: i for i, a in enumerate(_ACTS)}


_ACT_C = {
    "sigmoid": ("const double s0 = 1.0 / (1.0 + exp(-a));", "const double s1 = s0 * (1.0 - s0);",
                "const double s2 = s1 * (1.0 - 2.0 * s0);"),
    "tanh": ("const double s0 = tanh(a);", "const double s1 = 1.0 - s0 * s0;",
             "const double s2 = -2.0 * s0 * s1;"),
    "linear": ("const double s0 = a;", "const double s1 = 1.0;", "const double s2 = 0.0;"),
    "softplus": ("const double sg = 1.0 / (1.0 + exp(-a)); const double s0 = log(1.0 + exp(a));",
                 "const double s1 = sg;", "const double s2 = sg * (1.0 - sg);"),
    "exponential": ("const double s0 = exp(a);", "const double s1 = s0;", "const double s2 = s0;"),
    "gaussian": ("const double s0 = exp(-a * a);", "const double s1 = -2.0 * a * s0;",
                 "const double s2 = (4.0 * a * a - 2.0) * s0;"),
}


def _emit_network(nid: int, x: List[str], members: Dict[tuple, Expr], gp: str,
                  names: Dict[int, str], indent: str) -> List[str]:
    """One loop over the hidden units computing the used value/derivative entries."""
    net = _NETWORKS[nid]
    T = f"ANN{nid}"
    nin, H = net.n_in, net.H
    d1 = sorted(i for (k, i, _) in members if k == "d")
    d2 = sorted((i, j) for (k, i, j) in members if k == "dd")
    need_v = ("v", -1, -1) in members
    L = []
    if need_v:
        L.append(f"double {gp}v = {_c_literal(net.b2)};")
    L += [f"double {gp}g{i} = 0.0;" for i in d1]
    L += [f"double {gp}h{i}_{j} = 0.0;" for i, j in d2]
    L.append("#pragma unroll 4")
    L.append(f"for (int j = 0; j < {H}; ++j) {{")
    pre = " + ".join([f"{T}_B1[j]"] + [f"({x[i]}) * {T}_W1T[j * {nin} + {i}]" for i in range(nin)
                                        if np.any(net.W1[i] != 0.0)])
    L.append(f"  const double a = {pre};")
    acts = _ACT_C[net.act]
    L.append("  " + acts[0])
    L.append(f"  const double w = {T}_W2[j];")
    if need_v:
        L.append(f"  {gp}v += w * s0;")
    if d1:
        L.append("  " + acts[1])
        L.append("  const double c1 = w * s1;")
        L += [f"  {gp}g{i} += c1 * {T}_W1T[j * {nin} + {i}];" for i in d1]
    if d2:
        if not d1:
            L.append("  " + acts[1])
        L.append("  " + acts[2])
        L.append("  const double c2 = w * s2;")
        L += [f"  {gp}h{i}_{j} += c2 * ({T}_W1T[j * {nin} + {i}] * {T}_W1T[j * {nin} + {j}]);" for i, j in d2]
    L.append("}")
    for (k, i, j), node in members.items():
        names[node.uid] = f"{gp}v" if k == "v" else (f"{gp}g{i}" if k == "d" else f"{gp}h{i}_{j}")
    return [indent + l for l in L]


def network_tables(net_ids) -> List[str]:
    """``__constant__`` weight tables of the networks (W1 transposed: [H][n_in])."""
    out = []
    for nid in sorted(net_ids):
        net = _NETWORKS[nid]
        w1t = ", ".join(_c_literal(v) for v in net.W1.T.reshape(-1))
        b1 = ", ".join(_c_literal(v) for v in net.b1)
        w2 = ", ".join(_c_literal(v) for v in net.w2)
        out += [f"__constant__ double ANN{nid}_W1T[{net.H * net.n_in}] = {{{w1t}}};",
                f"__constant__ double ANN{nid}_B1[{net.H}] = {{{b1}}};",
                f"__constant__ double ANN{nid}_W2[{net.H}] = {{{w2}}};"]
    return out


def _c_op(op: str, a: List[str]) -> str:
    if op == "add":
        return f"{a[0]} + {a[1]}"
    if op == "sub":
        return f"{a[0]} - {a[1]}"
    if op == "mul":
        return f"{a[0]} * {a[1]}"
    if op == "div":
        return f"{a[0]} / {a[1]}"
    if op == "neg":
        return f"-({a[0]})"
    if op == "sq":
        return f"{a[0]} * {a[0]}"
    if op == "pow":
        return f"pow({a[0]}, {a[1]})"
    if op in ("exp", "log", "sqrt", "tanh", "sin", "cos", "fabs"):
        return f"{op}({a[0]})"
    if op == "fmax":
        return f"fmax({a[0]}, {a[1]})"
    if op == "fmin":
        return f"fmin({a[0]}, {a[1]})"
    if op == "lt":
        return f"(({a[0]}) < ({a[1]}) ? 1.0 : 0.0)"
    if op == "le":
        return f"(({a[0]}) <= ({a[1]}) ? 1.0 : 0.0)"
    if op == "eq":
        return f"(({a[0]}) == ({a[1]}) ? 1.0 : 0.0)"
    if op == "ne":
        return f"(({a[0]}) != ({a[1]}) ? 1.0 : 0.0)"
    if op == "if_else":
        return f"(({a[0]}) != 0.0 ? ({a[1]}) : ({a[2]}))"
    raise NotImplementedError(op)
