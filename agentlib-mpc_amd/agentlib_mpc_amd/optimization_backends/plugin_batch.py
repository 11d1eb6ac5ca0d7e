"""Device-resident inputs behind the plugin API's batched solve.

``MI355XBackend.solve_batch`` is the drop-in for ``OptimizationBackend.solve`` of every
agent of a fleet (`core/casadi_backend.py:133-139`): each call hands over one dict of
``MPCVariable`` per agent, which the reference samples onto the NLP grids
(`core/casadi_backend.py:141-253`), maps to the NLP vectors (`core/discretization.py:
277-348`) and warm-starts from the agent's previous optimum (`:212-251`).  Re-marshalling
every agent's dict into fresh [n, nw] host arrays and copying them to the GPU on every
call costs an order of magnitude more than the kernel at fleet sizes.

:class:`ResidentBatch` keeps the kernel's inputs in HBM between calls and, per call,

* reads every (variable, attribute) the marshalling needs in ONE native pass over the
  agents (``csrc/mpcx_pyread.c``: dict lookup, attribute lookup, float unpack into one
  buffer; Python iterators cost ~90 ns per read, 3-6 ms per 4096-agent call, more than
  the kernel); a variable whose instance dict has not changed since the last call (the
  dict's version tag) costs no lookups at all; lists, series and other trajectories take
  the sampling path of
  :class:`~agentlib_mpc_amd.optimization_backends.problem.BatchMarshal`, with the same
  errors for empty values and non-``MPCVariable`` inputs);
* uploads only the columns whose values changed since the last call and scatters them
  on the device into the parameter / bound columns the reference layout gives them
  (``GroupLayout.index``), then re-applies the bounds and guesses taken from parameters
  (the fixed ``x_0 = initial state``);
* keeps the solution in place as the next call's initial guess (the reference's one
  remembered optimum per backend, `core/discretization.py:221-223`); agents whose last
  solution holds NaN restart cold, as the reference's guess logic would.

The per-agent :class:`Results` are built on access from a snapshot of the values read
in that call (arrays that later calls never modify), so results stay valid after the
next solve.  Only problems solved in the reference layout take this path (lifted NARX /
MHE stage forms re-marshal on the host).
"""

from __future__ import annotations

import itertools
import operator
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from agentlib_mpc_amd.optimization_backends.problem import BatchMarshal

#: batches of at most this many agents update their inputs on the host and upload them in
#: one copy; larger ones scatter the changed columns on the device
SMALL_BATCH = 64


def _values(vs, attr, n):
    """(n,) float array of one attribute over the agents, or None if not all numbers
    (numpy reads None as NaN: NaN entries take the checked path too)."""
    try:
        arr = np.fromiter(map(operator.attrgetter(attr), vs), dtype=np.float64, count=n)
    except (TypeError, ValueError):
        return None
    return None if np.isnan(arr).any() else arr


class RowSource:
    """Reference-layout (p, sampled lbw, sampled ubw) rows of single agents, rebuilt from the
    values one call read (for :class:`~.problem.FleetResults`)."""

    def __init__(self, state: "ResidentBatch", snapshot: Dict[tuple, object]):
        self.state = state
        self.snapshot = snapshot

    def rows(self, i: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        st = self.state
        p, ls, us = st.base_p.copy(), st.base_ls.copy(), st.base_us.copy()
        dst = {"p": p, "ls": ls, "us": us}
        for key, cols in st.targets.items():
            val = self.snapshot[key]
            for arr_key, c, g in cols:
                v = val[g] if isinstance(val, dict) else val
                dst[arr_key][c] = v[i] if v.ndim == 1 else v[i, :len(c)]
        return p, ls, us


class MirrorRows:
    """:class:`RowSource` of a small batch: the host mirrors already hold every agent's
    reference-layout p and sampled bounds after :meth:`ResidentBatch.update` (the same values
    RowSource rebuilds from the read columns), copied at solve time."""

    def __init__(self, p: np.ndarray, ls: np.ndarray, us: np.ndarray):
        self.p, self.ls, self.us = p, ls, us

    def rows(self, i: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        return self.p[i].copy(), self.ls[i].copy(), self.us[i].copy()


def _has_nan(val) -> bool:
    """NaN in a read column (an (n,) array, or {grid: samples})."""
    if isinstance(val, np.ndarray):
        return bool(np.isnan(val).any()) if val.dtype.kind == "f" else False
    return any(np.isnan(np.asarray(a, dtype=np.float64)).any() for a in val.values())


class ResidentBatch:
    """Resident NLP inputs of one batch size of one backend (reference layout == kernel
    layout)."""

    def __init__(self, prob, native, batch_vars: Sequence[dict], now: float, device):
        import torch

        self.torch = torch
        self.prob, self.native = prob, native
        m: BatchMarshal = prob.marshal
        self.marshal = m
        self.n = n = len(batch_vars)
        self.dev = device
        # (ref, attr) -> [(array key, reference columns, group id)]; one group id per
        # (group, grid) so list / series values are sampled per grid
        self.targets: Dict[tuple, List[tuple]] = {}
        self.grids: Dict[int, list] = {}
        gid = 0
        for name, grid, rows, index in m.pars:
            if index is None:
                continue
            self.grids[gid] = grid
            for i, ref, _ in rows:
                if ref is not None:
                    self.targets.setdefault((ref, "value"), []).append(("p", index[i], gid))
            gid += 1
        for name, grid, rows, index in m.vars:
            if index is None:
                continue
            self.grids[gid] = grid
            for i, ref, _, _ in rows:
                if ref is not None:
                    self.targets.setdefault((ref, "lb"), []).append(("ls", index[i], gid))
                    self.targets.setdefault((ref, "ub"), []).append(("us", index[i], gid))
            gid += 1
        # every ref the host marshalling reads (also groups without grid points: validated)
        self.refs: Dict[str, List[str]] = {}
        for name, grid, rows, index in m.pars:
            for i, ref, _ in rows:
                if ref is not None:
                    self.refs.setdefault(ref, [])
                    if "value" not in self.refs[ref]:
                        self.refs[ref].append("value")
        for name, grid, rows, index in m.vars:
            for i, ref, _, _ in rows:
                if ref is not None:
                    lst = self.refs.setdefault(ref, [])
                    for at in ("lb", "ub"):
                        if at not in lst:
                            lst.append(at)
        from agentlib_mpc_amd.runtime.native import load_pyread

        self.pyread = load_pyread()
        # the reader's numbers of the last call, per (agent, variable), reused while the agent's
        # mapping and the variable's instance dict are unchanged (csrc/mpcx_pyread.c)
        self._read_cache = self.pyread.new_cache()
        self.specs = None
        # full marshal once: device arrays, template rows, the values of this call
        p, lbw, ubw, w0, (ls, us) = m.inputs(batch_vars, now, None, return_sampled_bounds=True)
        self.base_p, self.base_ls, self.base_us = p[0].copy(), ls[0].copy(), us[0].copy()
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(device)  # noqa: E731
        from agentlib_mpc_amd.runtime.native import STATS_BYTES

        # P, L, U, W, stats: contiguous blocks of ONE device buffer, so that a small batch uploads
        # all of its inputs with one copy and reads the solution and the stats back with one
        st_words = -(-n * STATS_BYTES // 8)
        sizes = [p.size, lbw.size, ubw.size, w0.size, st_words]
        self.BUF = torch.zeros(sum(sizes), dtype=torch.float64, device=device)
        offs = np.concatenate([[0], np.cumsum(sizes)])
        views = [self.BUF[offs[i]:offs[i + 1]].view(a.shape) for i, a in enumerate((p, lbw, ubw, w0))]
        self.P, self.L, self.U, self.W = views
        self.ST = self.BUF[offs[4]:].view(torch.uint8)[:n * STATS_BYTES]
        self._out_off = int(offs[3])  # W and the stats: the tail the solve writes
        self._buf_in = self.BUF[:offs[4]]  # what an upload writes
        self._buf_in.copy_(torch.from_numpy(np.concatenate([a.ravel() for a in (p, lbw, ubw, w0)])))
        self.LS, self.US = T(ls), T(us)  # sampled bounds (before the parameter overrides)
        # small batches (the reference's one agent per process): the inputs are kept on the
        # host too and updated there (numpy), then uploaded in one copy -- a handful of device
        # scatters costs ~20 us of launch overhead each, more than uploading a few KB
        self.small = n <= SMALL_BATCH
        if self.small:
            pin = device.type == "cuda"
            self.hbuf_t = torch.empty(sum(sizes), dtype=torch.float64, pin_memory=pin)
            self.hbuf = self.hbuf_t.numpy()
            self._h2d = None  # event after the last upload (the host mirrors are its source)
            self.hP, self.hL, self.hU, self.hW = [self.hbuf[offs[i]:offs[i + 1]].reshape(a.shape)
                                                  for i, a in enumerate((p, lbw, ubw, w0))]
            self.hbuf[:] = self.BUF.cpu().numpy()
            self._hbuf_in = self.hbuf_t[:offs[4]]
            self.hLS, self.hUS = ls.copy(), us.copy()
            self.over_h = {k: (c, q) for k, (c, q) in m.over.items() if c.size}
        self.idx = {}
        for key, cols in self.targets.items():
            for _, c, _ in cols:
                self.idx.setdefault(c.tobytes(), torch.as_tensor(c, device=device))
        self.over = {k: (torch.as_tensor(c, device=device), torch.as_tensor(q, device=device))
                     for k, (c, q) in m.over.items() if c.size}
        self._prev_buf = None
        self._cold_plan = None
        self._mid_cache = None  # (sampled bounds of the midpoint columns, their cold guess)
        self._unchanged = set()
        self.last: Dict[tuple, object] = self.read(batch_vars, now)
        self.cold_rows: Optional[np.ndarray] = None
        self.lam_g = torch.empty((n, prob.nlp.kernel_ng), dtype=torch.float64, device=device)
        self._launch = None
        if self.small and device.type == "cuda":
            self._pin_out = torch.empty(self.BUF.numel() - self._out_off, dtype=torch.float64, pin_memory=True)
        self._roundtrip = None

    # -- reading the agents' variables ---------------------------------------------------
    def read(self, batch_vars: Sequence[dict], now: float) -> Dict[tuple, object]:
        """Values of every (ref, attr) over the agents: an (n,) array when every agent holds a
        number, else {group id: (n, G) samples} (sampling path, reference errors).

        The numbers are read by ONE pass of the native reader over the agents
        (``csrc/mpcx_pyread.c``); the columns it cannot take (non-numbers, NaN) and a
        variable type without ``interpolation_method`` go through the Python path below,
        in variable order, so errors come out as the reference's, in its order."""
        n, m = self.n, self.marshal
        if self.specs is None:
            self.specs = [(ref, tuple(attrs), "value" in attrs) for ref, attrs in self.refs.items()]
            self.n_cols = sum(len(a) for _, a, _ in self.specs)
            self._col_keys = [(ref, attr) for ref, attrs, _ in self.specs for attr in attrs]
        if not isinstance(batch_vars, list):
            batch_vars = list(batch_vars)
        buf = np.empty((self.n_cols, n), dtype=np.float64)
        try:
            status, bad = self.pyread.read_columns(batch_vars, self.specs, buf, self._read_cache)
        except KeyError:  # a variable missing: the Python path raises it in the reference's order
            return self._read_python(batch_vars, now, self.refs)
        prev = self._prev_buf
        if bad < 0 and not status.strip(b"\x00"):
            # every column numeric (the usual case): the column keys in one zip, the unchanged
            # columns from one vectorised comparison
            self._prev_buf = buf
            if prev is not None and prev.shape == buf.shape:
                self._unchanged = set(itertools.compress(self._col_keys, ~np.any(buf != prev, axis=1)))
            else:
                self._unchanged = set()
            return dict(zip(self._col_keys, buf))
        out = {}
        c = 0
        slow = {}
        for s, (ref, attrs, _) in enumerate(self.specs):
            if s == bad:
                slow[ref] = attrs  # raises the reference's TypeError below
                break
            for attr in attrs:
                if status[c] == 0:
                    out[(ref, attr)] = buf[c]
                else:
                    slow.setdefault(ref, ())
                    slow[ref] += (attr,)
                c += 1
        # numeric columns unchanged since the last read, in one vectorised comparison (the
        # per-column comparisons were a sixth of a single agent's host time)
        self._unchanged = set()
        if prev is not None and prev.shape == buf.shape:
            same = ~np.any(buf != prev, axis=1)
            c = 0
            for ref, attrs, _ in self.specs:
                for attr in attrs:
                    if same[c] and status[c] == 0:
                        self._unchanged.add((ref, attr))
                    c += 1
        self._prev_buf = buf
        if slow:
            out.update(self._read_python(batch_vars, now, slow))
        return out

    def _same(self, key, val, old) -> bool:
        """Column ``key`` read the same values as at the last call."""
        if key in self._unchanged and isinstance(old, np.ndarray):
            return True
        return (isinstance(val, np.ndarray) and isinstance(old, np.ndarray) and val.shape == old.shape
                and np.array_equal(val, old)) or (
            isinstance(val, dict) and isinstance(old, dict) and val.keys() == old.keys()
            and all(np.array_equal(val[g], old[g]) for g in val))

    def _read_python(self, batch_vars, now, refs) -> Dict[tuple, object]:
        n, m = self.n, self.marshal
        out = {}
        for ref, attrs in refs.items():
            vs = list(map(operator.itemgetter(ref), batch_vars))
            if "value" in attrs:  # one object per type, as BatchMarshal.inputs checks
                for v in dict(zip(map(type, vs), vs)).values():
                    if not hasattr(v, "interpolation_method"):
                        raise TypeError(
                            f"The variable {ref} does not have an interpolationmethod. All Variables "
                            "used in MPC need to be of type MPCVariable (subclass of AgentVariable).")
            for attr in attrs:
                arr = _values(vs, attr, n)
                if arr is not None:
                    out[(ref, attr)] = arr
                    continue
                vals = list(map(operator.attrgetter(attr), vs))
                if attr == "value" and any(v is None for v in vals):
                    raise ValueError(f"Input for variable {ref} is empty. Cannot solve optimization problem.")
                meth = (lambda a: vs[a].interpolation_method) if attr == "value" else \
                    (lambda a: getattr(vs[a], "interpolation_method", "linear"))
                per = {}
                for _, _, g in self.targets.get((ref, attr), []):
                    if g not in per:
                        per[g] = m._column(vals, self.grids[g], now, meth)
                out[(ref, attr)] = per
        return out

    # -- one call ------------------------------------------------------------------------
    def update(self, batch_vars: Sequence[dict], now: float) -> Dict[tuple, object]:
        """Read the agents' variables, upload what changed, re-apply the parameter-derived
        bounds and guesses; returns the snapshot of the values read."""
        torch = self.torch
        cur = self.read(batch_vars, now)
        if self.small:
            return self._update_host(batch_vars, now, cur)
        dst = {"p": self.P, "ls": self.LS, "us": self.US}
        changed = nan_in = False
        for key, val in cur.items():
            old = self.last.get(key)
            if self._same(key, val, old):
                cur[key] = old  # keep the array already referenced by earlier snapshots
                continue
            changed = True
            nan_in |= _has_nan(val)
            if isinstance(val, np.ndarray):
                dv = torch.from_numpy(val).to(self.dev, non_blocking=True)
            else:
                dvs = {g: torch.from_numpy(np.ascontiguousarray(a)).to(self.dev, non_blocking=True)
                       for g, a in val.items()}
            for arr_key, c, g in self.targets.get(key, []):
                ix = self.idx[c.tobytes()]
                if isinstance(val, np.ndarray):
                    dst[arr_key][:, ix] = dv[:, None].expand(-1, ix.numel())
                else:
                    dst[arr_key][:, ix] = dvs[g][:, :ix.numel()]
        if changed:
            self.L.copy_(self.LS)
            self.U.copy_(self.US)
            for k, arr in (("lb", self.L), ("ub", self.U)):
                if k in self.over:
                    c, q = self.over[k]
                    arr[:, c] = self.P[:, q]
        if nan_in and bool(torch.isnan(self.P).any() | torch.isnan(self.L).any() | torch.isnan(self.U).any()):
            self._reject_nan()
        if "guess" in self.over:
            c, q = self.over["guess"]
            self.W[:, c] = self.P[:, q]
        if self.cold_rows is not None and self.cold_rows.size:
            rows = [batch_vars[i] for i in self.cold_rows]
            _, _, _, w0 = self.marshal.inputs(rows, now, None)
            self.W[torch.as_tensor(self.cold_rows, device=self.dev)] = torch.from_numpy(w0).to(self.dev)
            self.cold_rows = None
        self.last = cur
        return cur

    def _update_host(self, batch_vars, now, cur):
        """:meth:`update` of a small batch: the same scatters on the host mirrors, one upload."""
        if self._h2d is not None:
            self._h2d.synchronize()  # the last upload has read the mirrors
        dst = {"p": self.hP, "ls": self.hLS, "us": self.hUS}
        changed = nan_in = False
        last, unch = self.last, self._unchanged
        for key, val in cur.items():
            old = last.get(key)
            if (key in unch and isinstance(old, np.ndarray)) or self._same(key, val, old):
                cur[key] = old
                continue
            changed = True
            nan_in |= _has_nan(val)
            for arr_key, c, g in self.targets.get(key, []):
                if isinstance(val, np.ndarray):
                    dst[arr_key][:, c] = val[:, None]
                else:
                    dst[arr_key][:, c] = val[g][:, :c.size]
        if changed:
            self.hL[:] = self.hLS
            self.hU[:] = self.hUS
            for k, arr in (("lb", self.hL), ("ub", self.hU)):
                if k in self.over_h:
                    c, q = self.over_h[k]
                    arr[:, c] = self.hP[:, q]
        if nan_in and (np.isnan(self.hP).any() or np.isnan(self.hL).any() or np.isnan(self.hU).any()):
            self._reject_nan()
        if "guess" in self.over_h:
            c, q = self.over_h["guess"]
            self.hW[:, c] = self.hP[:, q]
        if self.cold_rows is not None and self.cold_rows.size:
            self.hW[self.cold_rows] = self._cold_guess(self.cold_rows)
            self.cold_rows = None
        if self.dev.type != "cuda":
            self._buf_in.copy_(self._hbuf_in)  # on the GPU, solve() stages the upload
        self.last = cur
        return cur

    def _reject_nan(self):
        """A NaN reached the parameters or the bounds: the host path's error
        (``BatchMarshal.assemble``: 'incomplete NLP inputs'), and nothing is launched.  The
        snapshot is dropped so that the next call re-applies every column (the NaN values
        are already scattered into the resident arrays)."""
        self.last = {}
        raise ValueError("incomplete NLP inputs (NaN in parameters or bounds)")

    def _cold_guess(self, rows) -> np.ndarray:
        """The cold-start guess of some agents (``BatchMarshal.assemble`` with no previous
        optimum, `core/discretization.py:212-245`) from the host mirrors: states tiled from
        their measured initial value, other variables at the midpoint of their sampled bounds
        (infinite -> 0), then the guesses taken from parameters.  The column maps are built once
        (three gathers per call: the per-variable loop cost ~0.1 ms, a fifth of a single agent's
        solve)."""
        if self._cold_plan is None:
            m = self.marshal
            dst_a, src_a, mid = [], [], []
            for name, grid, _, index in m.vars:
                if index is None:
                    continue
                flat = index.ravel()
                if name in m.initial:
                    cols = m.initial[name][:, -1]
                    dst_a.append(flat)
                    src_a.append(np.repeat(cols[:, None], len(grid), axis=1).reshape(-1))
                else:
                    mid.append(flat)
            cat = lambda parts: np.concatenate(parts).astype(np.int64) if parts else np.zeros(0, np.int64)  # noqa
            self._cold_plan = (cat(dst_a), cat(src_a), cat(mid))
        dst_a, src_a, mid = self._cold_plan
        if len(rows) == self.n:  # every agent (a cold restart): no row gathers
            P, LS, US = self.hP, self.hLS, self.hUS
        else:
            P, LS, US = self.hP[rows], self.hLS[rows], self.hUS[rows]
        g = np.zeros((len(rows), self.hW.shape[1]))
        g[:, dst_a] = P[:, src_a]
        lo, hi = LS[:, mid], US[:, mid]
        key = (lo.tobytes(), hi.tobytes())
        if self._mid_cache is not None and self._mid_cache[0] == key:
            v = self._mid_cache[1]  # the same sampled bounds as at the last cold start
        else:
            with np.errstate(invalid="ignore"):
                v = 0.5 * (lo + hi)
            bad = ~np.isfinite(v)
            if bad.any():  # nan_to_num(posinf=0, neginf=-0)
                v[bad] = np.where(v[bad] < 0, -0.0, 0.0)
            self._mid_cache = (key, v)
        g[:, mid] = v
        if "guess" in self.over_h:
            c, q = self.over_h["guess"]
            g[:, c] = P[:, q]
        return g if np.isfinite(g).all() else np.nan_to_num(g)

    # -- warm starts keyed by agent (MI355XBackend.solve_batch agent_ids) ---------------
    def permute_warm_starts(self, src: np.ndarray):
        """Entry i takes the warm start of the previous call's slot src[i] (-1: cold start,
        applied by the next update).  Same batch size; the inputs are re-read by update()
        (a column whose per-entry values moved differs from the snapshot and is re-applied).
        Pending cold starts (slots whose last solve came back NaN, in the OLD numbering) move
        with their agents: entry i is cold when src[i] < 0 or src[i] was cold."""
        src = np.asarray(src, np.int64)
        if np.array_equal(src, np.arange(self.n)):
            return
        was_cold = self.cold_rows if self.cold_rows is not None else np.zeros(0, np.int64)
        self.cold_rows = None
        cold_src = np.isin(src, was_cold)
        hit = np.flatnonzero((src >= 0) & ~cold_src)
        cold = np.flatnonzero((src < 0) | cold_src)
        if hit.size:
            rows = self.torch.as_tensor(src[hit], device=self.dev)
            dst = self.torch.as_tensor(hit, device=self.dev)
            self.W[dst] = self.W[rows].clone()
            if self.small:
                if self._h2d is not None:
                    self._h2d.synchronize()
                self.hW[hit] = self.hW[src[hit]].copy()
        self._mark_cold(cold)

    def adopt_warm_starts(self, old: "ResidentBatch", src: np.ndarray):
        """A new batch (new size): entry i takes the warm start of slot src[i] of the old
        batch (-1, or an old slot whose last solve came back NaN: keeps its cold-start guess)."""
        src = np.asarray(src, np.int64)
        if old.cold_rows is not None and old.cold_rows.size:
            src = np.where(np.isin(src, old.cold_rows), -1, src)
        hit = np.flatnonzero(src >= 0)
        if not hit.size:
            return
        rows = self.torch.as_tensor(src[hit], device=self.dev)
        self.W[self.torch.as_tensor(hit, device=self.dev)] = old.W[rows].to(self.dev)
        if self.small:
            self.hW[hit] = old.W[rows].cpu().numpy()

    def _mark_cold(self, rows: np.ndarray):
        if rows.size:
            prev = self.cold_rows if self.cold_rows is not None else np.zeros(0, np.int64)
            self.cold_rows = np.union1d(prev, rows).astype(np.int64)

    def row_source(self, snapshot):
        """What :class:`~.problem.FleetResults` rebuilds each agent's reference-layout rows
        from: the host mirrors of a small batch (copied now), else the call's read columns."""
        if self.small:
            return MirrorRows(self.hP.copy(), self.hLS.copy(), self.hUS.copy())
        return RowSource(self, snapshot)

    def restart_cold(self):
        """Every agent's next guess is the cold-start guess (no remembered optimum)."""
        self.cold_rows = np.arange(self.n)

    def solve(self):
        """Launch on the resident arrays (the solution replaces the guess in place); returns
        (w, raw stats) on the host."""
        torch = self.torch
        if self.small:
            # ONE native call: the host mirrors uploaded from pinned memory, the solve, solution and
            # stats read back into a persistent pinned buffer, the wait (as separate torch copies,
            # events and a launch: ~25 us more per call, a twentieth of a single agent's solve)
            if self._roundtrip is None:
                self._roundtrip = self.native.bind_staged(self.P, self.L, self.U, self.W, self.lam_g, self.ST,
                                                          self._hbuf_in, self._buf_in, self._pin_out,
                                                          self.BUF[self._out_off:])
            self._roundtrip()
            out = self._pin_out.numpy()
            nw = self.hW.size
            w = out[:nw].reshape(self.hW.shape).copy()
            raw = out[nw:].view(np.uint8)[:self.ST.numel()].copy()
            self.hW[:] = w  # the next call's warm start (uploaded with the inputs)
        else:
            if self._launch is None:  # the buffers are resident: checked once, pointers pre-bound
                self._launch = self.native.bind(self.P, self.L, self.U, self.W, lam_g=self.lam_g, stats=self.ST)
            self._launch()
            w = torch.empty((self.n, self.W.shape[1]), dtype=torch.float64, pin_memory=True)
            w.copy_(self.W, non_blocking=True)
            raw = self.ST.cpu().numpy()  # synchronises (w is complete too: same stream)
            w = w.numpy()
        with np.errstate(invalid="ignore"):
            bad = np.flatnonzero(np.isnan(w.sum(axis=1)))
        self.cold_rows = bad if bad.size else None
        return w, raw
