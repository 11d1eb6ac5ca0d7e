"""Fleet ADMM drivers: coordinated (consensus/exchange) and decentralised ADMM over
device-resident fleets of agents, partitioned by agent across GPUs.

The reference runs one agentlib module per agent and moves trajectories between
them as JSON messages; every agent solves its own NLP through ``backend.solve``
(SURVEY §3.C/§3.D).  Here all agents of one problem structure ("class") are
solved by ONE batched kernel launch, their coupling trajectories never leave
HBM, and the consensus/exchange arithmetic runs as HIP kernels.  Semantics
follow, step for step:

* coordinated ADMM — ``ADMMCoordinator._fast_process``
  (`modules/dmpc/admm/admm_coordinator.py:259-321`): mean update from the last
  locals, shift (:323-337), then per iteration trigger → local solves
  (``CoordinatedADMM.optimize``, `admm_coordinated.py:133-193`) → mean update →
  multiplier update (:339-347) → residual check with optional penalty variation
  (:354-435, :467-479); ρ reset after the round (:665).
* decentralised ADMM — ``LocalADMM.process`` (`modules/dmpc/admm/admm.py:873-937`):
  shift and send locals and multipliers (:329-375), mean / mean-diff from the
  shifted locals, then ``max_iterations`` × (solve → mean → multiplier update).

Blocks: the participation graph (agents — aliases) splits into connected
components, each the counterpart of ONE reference coordinator (e.g. the
4-room + air-handler blocks of a scaled C2 fleet).  Coordinated runs keep a
stopping test, a penalty parameter and an iteration count per block and freeze
a block (no solves, no updates) once it has converged, exactly as that block's
own ``ADMMCoordinator`` would stop (`admm_coordinator.py:284-309`).

Multi-GPU: one process per GPU, each holding a contiguous slice of every
class's agents.  Aliases whose participants live on several ranks are "global
groups"; their per-(group, t) moments, the residual totals of the blocks spanning ranks and
the coordinated loop's count of blocks still active (one control double) travel in ONE
``all_reduce(SUM)`` per ADMM iteration (`include/mpcx.h`, ``mpcx_admm_reduce_count``).  No
other collective is on the data path.
"""

from __future__ import annotations

import contextlib
import dataclasses
import math
import os
import sys
import time
from typing import Dict, List, Optional, Sequence, Union

import numpy as np

from agentlib_mpc_amd.data_structures import admm_datatypes as adt
from agentlib_mpc_amd.runtime.native import ADMM_CONTROL, ADMM_TOTALS, STATS_BYTES, admm_reduce_count, dedicated_streams

CONSENSUS = "consensus"
EXCHANGE = "exchange"
NMOM = 5
_ITER_WORD = 12  # int32 index of mpcx_stats.iter_count
_STATUS_WORD = 13  # int32 index of mpcx_stats.status (6 doubles + iter_count)


@dataclasses.dataclass
class Slot:
    """One coupling of one class: where its trajectory lives in w and p."""

    name: str
    kind: str
    aliases: List[str]
    initial: np.ndarray           # [n] initial value of the local trajectory
    w_cols: np.ndarray            # [T] columns of the local trajectory in w
    mean_cols: np.ndarray         # [T] columns of the mean (consensus) / mean diff (exchange) in p
    mult_cols: np.ndarray         # [T] columns of the multiplier in p


def _local_cols(lay, comp: int) -> List[int]:
    """w columns of ``Results[name]`` (first occurrence of every grid time >= 0)."""
    seen, cols = set(), []
    for j, t in enumerate(lay.grid):
        if t >= 0 and t not in seen:
            seen.add(t)
            cols.append(lay.columns[j][comp])
    return cols


class FleetClass:
    """All agents (on this rank) that share one problem structure.

    ``backend`` is a set-up :class:`MI355XADMMBackend`; ``inputs`` the cold-start
    NLP inputs ``(p, lbw, ubw, w0)`` as [n, .] arrays (e.g. from
    :func:`~agentlib_mpc_amd.optimization_backends.problem.fleet_nlp_inputs`).
    ``aliases`` maps a coupling/exchange variable name to its alias — one string
    for all agents or one per agent (default: the variable name).  ``initial``
    maps it to the initial local value (scalar or per agent), which the reference
    takes from the module config (`admm_coordinated.py:226-238`, `admm.py:700-780`).
    """

    def __init__(self, name: str, backend, inputs, aliases: Optional[Dict[str, Union[str, Sequence[str]]]] = None,
                 initial: Optional[Dict[str, Union[float, Sequence[float]]]] = None):
        self.name = name
        self.backend = backend
        prob = backend.problem
        nlp = prob.nlp
        self.lift = nlp.lift
        self.lbw_ref = np.ascontiguousarray(inputs[1], dtype=np.float64)
        # device arrays are in the kernel's stage order (== reference order unless lifted)
        p, lbw, ubw, w0 = (np.ascontiguousarray(a, dtype=np.float64) for a in prob.to_kernel(*inputs))
        self.p0, self.lbw, self.ubw, self.w0 = p, lbw, ubw, w0
        self.n = p.shape[0]
        sysm = backend.system
        aliases = aliases or {}
        initial = initial or {}
        self.slots: List[Slot] = []
        ref = backend.var_ref
        specs = [(c.name, CONSENSUS, c.mean, c.multiplier, "local_couplings", "global_couplings", "multipliers")
                 for c in getattr(ref, "couplings", [])]
        specs += [(c.name, EXCHANGE, c.mean_diff, c.multiplier, "local_exchange", "average_diff",
                   "exchange_multipliers") for c in getattr(ref, "exchange", [])]
        groups = {q.name: q for q in sysm.quantities}
        for name, kind, mean_name, mult_name, vg, mg, lg in specs:
            comp = groups[vg].full_names.index(name)
            w_cols = _local_cols(nlp.var_groups[vg], comp)
            mlay, llay = nlp.par_groups[mg], nlp.par_groups[lg]
            mean_cols = [c[groups[mg].full_names.index(mean_name)] for c in mlay.columns]
            mult_cols = [c[groups[lg].full_names.index(mult_name)] for c in llay.columns]
            if not (len(w_cols) == len(mean_cols) == len(mult_cols)):
                raise ValueError(f"{name}: trajectory lengths differ (local {len(w_cols)}, mean "
                                 f"{len(mean_cols)}, multiplier {len(mult_cols)})")
            if self.lift is not None:
                w_cols = self.lift.w_primary[np.asarray(w_cols)]
                mean_cols = [self._kernel_par(c) for c in mean_cols]
                mult_cols = [self._kernel_par(c) for c in mult_cols]
            al = aliases.get(name, name)
            al = [al] * self.n if isinstance(al, str) else list(al)
            if len(al) != self.n:
                raise ValueError(f"{name}: {len(al)} aliases for {self.n} agents")
            init = np.broadcast_to(np.asarray(initial.get(name, 0.0), float), (self.n,)).copy()
            self.slots.append(Slot(name, kind, al, init, np.asarray(w_cols, np.int32),
                                   np.asarray(mean_cols, np.int32), np.asarray(mult_cols, np.int32)))
        if not self.slots:
            raise ValueError(f"class {name}: backend has no couplings or exchange variables")
        self.rho_col = int(nlp.par_groups[sysm.penalty_factor.name].columns[0][0])
        if self.lift is not None:
            self.rho_col = self._kernel_par(self.rho_col)
        self.T = len(self.slots[0].w_cols)
        opts = backend.config.discretization_options
        self.horizon = int(opts.prediction_horizon)
        self.time_step = float(opts.time_step)
        self.coupling_grid = list(backend.coupling_grid)

    def _kernel_par(self, ref_col: int) -> int:
        """Kernel parameter column of a reference parameter that the stages read once."""
        hits = np.flatnonzero(self.lift.p_src == ref_col)
        if len(hits) != 1:
            raise ValueError(f"parameter {ref_col} appears {len(hits)} times in the kernel NLP")
        return int(hits[0])

    def to_kernel(self, p=None, lbw=None, ubw=None):
        """Reference-layout class inputs -> kernel layout (None passes through)."""
        if self.lift is None:
            return p, lbw, ubw
        if p is None or lbw is None or ubw is None:
            raise ValueError("lifted classes need p, lbw and ubw together")
        kp, klb, kub, _ = self.backend.problem.to_kernel(np.asarray(p), np.asarray(lbw), np.asarray(ubw),
                                                         np.asarray(lbw))
        return kp, klb, kub

    @property
    def native(self):
        return self.backend._native()


@dataclasses.dataclass
class IterationRecord:
    primal_residual: float
    dual_residual: float
    penalty: float                     # after the penalty variation (admm_coordinator.py:396-397)
    converged_solves: Optional[int] = None
    wall_time: Optional[float] = None  # seconds since the start of the round (:270, :400-402)


class _BlockRecords(Sequence):
    """Per-block residual histories of a coordinated round (``block_records[b]`` = block b's
    list of :class:`IterationRecord`), kept as one array row per iteration and expanded
    on access: building 1024 record objects per ADMM iteration cost about as much host
    time as the iteration's batched solves."""

    def __init__(self, n_blocks: int):
        self.n = n_blocks
        self._rows = []   # (prim, dual, rho, active, wall_time) per iteration

    def append(self, prim, dual, rho, active, wall_time):
        self._rows.append((np.array(prim, float), np.array(dual, float), np.array(rho, float),
                           np.array(active, bool), float(wall_time)))

    def __len__(self):
        return self.n

    def __getitem__(self, b):
        if isinstance(b, slice):
            return [self[i] for i in range(*b.indices(self.n))]
        if b < 0:
            b += self.n
        if not 0 <= b < self.n:
            raise IndexError(b)
        return [IterationRecord(float(p[b]), float(d[b]), float(r[b]), wall_time=t)
                for p, d, r, a, t in self._rows if a[b]]


_DEBUG = os.environ.get("MPCX_FLEET_DEBUG", "0") == "1"


class ADMMFleet:
    """Device-resident ADMM over fleets of agents (one or more classes).

    ``ops`` is the device backend (default :class:`~agentlib_mpc_amd.admm.ops.NativeADMMOps`);
    ``comm`` a ``torch.distributed`` process group (or ``None`` for one GPU / the
    default group when the default group is initialised and ``comm="default"``).
    """

    def __init__(self, classes: Sequence[FleetClass], device=None, ops=None, comm=None):
        import torch

        self.torch = torch
        self.classes = list(classes)
        if ops is None:
            from agentlib_mpc_amd.admm.ops import NativeADMMOps

            ops = NativeADMMOps()
        self.ops = ops
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.dist = None
        self.collective = None
        if comm is not None:
            import torch.distributed as dist

            self.dist = dist
            self.group = None if comm == "default" else comm
            self.world = dist.get_world_size(self.group)
            if self.world > 1:
                # the iteration's one all-reduce goes through the C ABI (mpcx_admm_allreduce, v14)
                from agentlib_mpc_amd.runtime.collective import Collective

                self.collective = Collective(dist, self.group, self.device)
        else:
            self.world = 1
        T = {c.T for c in self.classes}
        if len(T) != 1:
            raise ValueError(f"all coupling trajectories must have one length, got {sorted(T)}")
        self.T = T.pop()
        self._build_groups()
        self._allocate()
        self.history: List[IterationRecord] = []
        self.rounds = 0
        self._masked = False
        self._part = None      # per-class participation masks (host) of the current round
        self._blk_key = None   # last uploaded (penalties, freeze mask) of _set_blocks
        self.ROW_ON = None     # participation of the rows (device int32 [R + 1]) or None

    # ------------------------------------------------------------------ setup
    def _build_groups(self):
        kinds: Dict[str, str] = {}
        parts = []  # (alias, class idx, slot idx, agent idx)
        for ci, c in enumerate(self.classes):
            for si, s in enumerate(c.slots):
                for a, al in enumerate(s.aliases):
                    if kinds.setdefault(al, s.kind) != s.kind:
                        raise ValueError(f"alias {al!r} mixes consensus and exchange participants")
                    parts.append((al, ci, si, a))
        local_aliases = sorted(kinds)
        if self.world > 1:
            gathered = [None] * self.world
            self.dist.all_gather_object(gathered, sorted(kinds.items()), group=self.group)
            count: Dict[str, int] = {}
            all_kinds: Dict[str, str] = {}
            for lst in gathered:
                for al, k in lst:
                    count[al] = count.get(al, 0) + 1
                    if all_kinds.setdefault(al, k) != k:
                        raise ValueError(f"alias {al!r} mixes consensus and exchange participants")
            global_aliases = sorted(al for al, n in count.items() if n > 1)
            self.global_kinds = {al: all_kinds[al] for al in global_aliases}
        else:
            global_aliases = []
            self.global_kinds = {}
        gset = set(global_aliases)
        order = global_aliases + [al for al in local_aliases if al not in gset]
        self.n_global = len(global_aliases)
        self.aliases = order
        gid = {al: i for i, al in enumerate(order)}
        G = len(order)
        self.G = G
        kind_of = dict(self.global_kinds)
        kind_of.update(kinds)
        self.exchange_flags = np.array([1 if kind_of[al] == EXCHANGE else 0 for al in order], np.int32)
        parts.sort(key=lambda x: gid[x[0]])  # stable: class, slot, agent order inside a group
        counts = np.zeros(G, np.int64)
        rows = {}
        for r, (al, ci, si, a) in enumerate(parts):
            counts[gid[al]] += 1
            rows[(ci, si, a)] = r
        self._build_blocks(parts, order, gid)
        self.R = len(parts)
        self.gstart = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
        self.max_rows = int(counts.max()) if G else 0
        self.slot_rows = {}
        self.slot_groups = {}
        for ci, c in enumerate(self.classes):
            for si, s in enumerate(c.slots):
                self.slot_rows[(ci, si)] = np.array([rows[(ci, si, a)] for a in range(c.n)], np.int32)
                self.slot_groups[(ci, si)] = np.array([gid[al] for al in s.aliases], np.int32)

    def _build_blocks(self, parts, order, gid):
        """Connected components of the agent-alias participation graph: one block per
        reference coordinator.  Blocks that contain a global alias (participants on several
        ranks) are merged over the ranks and numbered first, identically on every rank
        (``n_global_blocks``); the rank-local blocks follow in local order.  Only the global
        blocks' residual totals travel in the all-reduce, so its length does not grow with
        the number of rank-local blocks."""
        parent = {al: al for al in order}

        def find(a):
            while parent[a] != a:
                parent[a] = parent[parent[a]]
                a = parent[a]
            return a

        def union(a, b):
            ra, rb = find(a), find(b)
            if ra != rb:
                parent[max(ra, rb)] = min(ra, rb)

        by_agent: Dict[tuple, List[str]] = {}
        for al, ci, si, a in sorted(parts, key=lambda x: (x[1], x[3], x[2])):  # class, agent, slot
            by_agent.setdefault((ci, a), []).append(al)
        seen: List[str] = []  # aliases in order of first appearance (class, agent)
        for als in by_agent.values():
            seen.extend(als)
            for al in als[1:]:
                union(als[0], al)
        gset = set(order[:self.n_global])
        comps: Dict[str, List[str]] = {}
        for al in list(dict.fromkeys(seen)) + [al for al in order if al not in set(seen)]:
            comps.setdefault(find(al), []).append(al)
        # global blocks: merge the components that share global aliases over the ranks
        gparent = {al: al for al in gset}

        def gfind(a):
            while gparent[a] != a:
                gparent[a] = gparent[gparent[a]]
                a = gparent[a]
            return a

        def gunion(a, b):
            ra, rb = gfind(a), gfind(b)
            if ra != rb:
                gparent[max(ra, rb)] = min(ra, rb)

        local_links = [sorted(al for al in c if al in gset) for c in comps.values()]
        local_links = [ln for ln in local_links if ln]
        links = local_links
        if self.world > 1:
            gathered = [None] * self.world
            self.dist.all_gather_object(gathered, local_links, group=self.group)
            links = [ln for lst in gathered for ln in lst]
        for ln in links:
            for al in ln:
                gparent.setdefault(al, al)
            for al in ln[1:]:
                gunion(ln[0], al)
        groots = sorted({gfind(al) for al in gparent})
        gbid = {r: i for i, r in enumerate(groots)}
        self.n_global_blocks = len(groots)
        bid_of_root: Dict[str, int] = {}
        nxt = self.n_global_blocks
        for root, c in comps.items():
            gl = [al for al in c if al in gset]
            if gl:
                bid_of_root[root] = gbid[gfind(gl[0])]
            else:
                bid_of_root[root] = nxt
                nxt += 1
        self._block_id = {al: bid_of_root[find(al)] for al in parent}
        self.n_blocks = max(nxt, 1)
        self.block_is_global = np.arange(self.n_blocks) < self.n_global_blocks
        self.block_of_group = np.array([self._block_id[al] for al in order], np.int32)
        self.block_aliases = [[] for _ in range(self.n_blocks)]
        for al in sorted(parent):
            self.block_aliases[self._block_id[al]].append(al)
        self.agent_blocks = {}
        for ci, c in enumerate(self.classes):
            blk = np.zeros(c.n, np.int32)
            for (cj, a), als in by_agent.items():
                if cj == ci:
                    blk[a] = self._block_id[als[0]]
            self.agent_blocks[ci] = blk

    def block_index(self, alias: str) -> int:
        """Block (coordinator) of an alias."""
        return self._block_id[alias]

    def _allocate(self):
        t = self.torch
        dev, f64, i32 = self.device, t.float64, t.int32
        T, G, R = self.T, self.G, max(self.R, 1)
        self.X = t.zeros((R + 1, T), dtype=f64, device=dev)      # local trajectories (+ scratch row R)
        self.LAMR = t.zeros((R, T), dtype=f64, device=dev)       # consensus multipliers per participant
        self.DIFF = t.zeros((R, T), dtype=f64, device=dev)       # exchange mean diffs per participant
        self.MEAN = t.zeros((max(G, 1), T), dtype=f64, device=dev)
        self.DMEAN = t.zeros((max(G, 1), T), dtype=f64, device=dev)
        self.GMULT = t.zeros((max(G, 1), T), dtype=f64, device=dev)  # exchange multiplier per alias
        self.EXCH = t.as_tensor(self.exchange_flags if G else np.zeros(1, np.int32), dtype=i32, device=dev)
        self.GSTART = t.as_tensor(self.gstart, dtype=i32, device=dev)
        self.S = NMOM * T + 1
        nb = self.n_blocks
        # [control][moments buffer]: the all-reduce range starts at the control double (the
        # coordinated loop's count of blocks still active), then the global groups' moments and
        # the totals of the blocks spanning ranks (numbered first), as the C ABI defines it
        # (include/mpcx.h mpcx_admm_reduce_count, v10); the kernels get the moments buffer
        self.MOMBUF = t.zeros(ADMM_CONTROL + self.ops.moments_size(max(G, 1), nb, T), dtype=f64, device=dev)
        self.CONTROL = self.MOMBUF[:ADMM_CONTROL]
        self.MOM = self.MOMBUF[ADMM_CONTROL:]
        self.totals_off = self.n_global * self.S
        self.reduce_len = admm_reduce_count(self.n_global, self.n_global_blocks, T) if self.world > 1 else 0
        if self.collective is not None:
            self.collective.bind(self.MOMBUF)
        #: all-reduces issued (the one collective per ADMM iteration; tests count them)
        self.n_collectives = 0
        # per-block coordinator state on the device: penalty, group freeze mask
        self.BLOCK_G = t.as_tensor(self.block_of_group if G else np.zeros(1, np.int32), dtype=i32, device=dev)
        self.RHO_B = t.zeros((nb, 1), dtype=f64, device=dev)
        self.RHO_G = t.zeros(max(G, 1), dtype=f64, device=dev)
        self.ACTIVE_G = t.ones(max(G, 1), dtype=i32, device=dev)
        self._rho_col = t.zeros(1, dtype=i32, device=dev)
        for ci, c in enumerate(self.classes):
            c.P = t.as_tensor(c.p0, device=dev).contiguous()
            c.LB = t.as_tensor(c.lbw, device=dev).contiguous()
            c.UB = t.as_tensor(c.ubw, device=dev).contiguous()
            c.W = t.as_tensor(c.w0, device=dev).contiguous()
            c.LAMG = t.zeros((c.n, c.backend.problem.nlp.kernel_ng), dtype=f64, device=dev)
            c.ST = t.zeros(c.n * STATS_BYTES, dtype=t.uint8, device=dev)
            c.BLOCK = t.as_tensor(self.agent_blocks[ci], dtype=i32, device=dev)
            c.ACTIVE = t.ones(c.n, dtype=i32, device=dev)
            c.RHO_COL = t.as_tensor(np.array([c.rho_col], np.int32), device=dev)
            c.dev_slots = []
            for si, s in enumerate(c.slots):
                c.dev_slots.append({
                    "w_cols": t.as_tensor(s.w_cols, dtype=i32, device=dev),
                    "mean_cols": t.as_tensor(s.mean_cols, dtype=i32, device=dev),
                    "mult_cols": t.as_tensor(s.mult_cols, dtype=i32, device=dev),
                    "rows": t.as_tensor(self.slot_rows[(ci, si)], dtype=i32, device=dev),
                    "groups": t.as_tensor(self.slot_groups[(ci, si)], dtype=i32, device=dev),
                })
        # initial local trajectories (registration, `admm_coordinator.py:528-560`;
        # `admm.py:356-375`): the configured value repeated over the coupling grid
        x0 = np.zeros((R, T))
        for ci, c in enumerate(self.classes):
            for si, s in enumerate(c.slots):
                x0[self.slot_rows[(ci, si)]] = s.initial[:, None]
        self.X[:R].copy_(t.as_tensor(x0, device=dev))
        # [converged solves, restoration-phase calls] of the round's batched solves
        self._counts = t.zeros(2, dtype=t.int64, device=dev)
        #: a list to record every iteration's local-solve (iter_count, status) per class (device
        #: copies, [n, 2] int32) -- the per-agent counterpart of the reference's per-solve stats;
        #: None (the default) records nothing
        self.solve_trace = None
        #: the classes' solves of an iteration on one HIP stream each (see _solve_all);
        #: MPCX_FLEET_STREAMS=0 keeps them on the caller's stream.  MPCX_FLEET_DEDICATED=1 gives each
        #: class stream a hardware queue of its own (C ABI v15): the classes' solves then overlap, but
        #: every launch of the iteration's main-stream kernels waits ~15 us more with three queues
        #: active, and the legs measured slower (r06/s11: C4 663 vs 755 it/s, C5 376 vs 420, C2
        #: level) -- so ordinary streams (sharing the runtime's queues) stay the default
        self.concurrent_classes = (dev.type == "cuda" and len(self.classes) > 1
                                   and os.environ.get("MPCX_FLEET_STREAMS", "1") != "0")
        if not self.concurrent_classes:
            self._class_streams = None
        elif os.environ.get("MPCX_FLEET_DEDICATED", "0") == "1":
            self._class_streams = dedicated_streams(len(self.classes), dev)
        else:
            self._class_streams = [t.cuda.Stream(device=dev) for _ in self.classes]
        self._ev_solve = t.cuda.Event() if self.concurrent_classes else None
        #: the lead class (most agents x NLP size) is issued first and the others wait for its
        #: pre-solve moves (see _solve_all); MPCX_FLEET_LEAD=0: every class starts at once
        size = [c.n * (c.P.shape[1] + c.W.shape[1]) for c in self.classes]
        self._lead = (int(np.argmax(size)) if self.concurrent_classes and os.environ.get("MPCX_FLEET_LEAD", "1") != "0"
                      else None)
        self._class_order = ([self._lead] + [i for i in range(len(self.classes)) if i != self._lead]
                             if self._lead is not None else list(range(len(self.classes))))
        self._ev_lead = t.cuda.Event() if self._lead is not None else None
        #: the lead class's solve on the caller's stream itself, the others on their class streams:
        #: the two overlap on two hardware queues (the class streams share one), and the iteration's
        #: small kernels keep their back-to-back dispatch -- C2 1076 / 931 -> 1203 / 1139 ADMM it/s,
        #: C4 level (r06/s12).  Not for a lead class whose agents fill a CU's LDS (4 per CU or fewer,
        #: the C5 zones: 434 / 414 -> 396 / 393): the others' workgroups then split its launch.
        #: MPCX_FLEET_LEAD_MAIN=1 / 0 forces it on / off
        lead_env = os.environ.get("MPCX_FLEET_LEAD_MAIN", "auto")
        if self._lead is None or lead_env == "0":
            self._lead_on_main = False
        elif lead_env == "1":
            self._lead_on_main = True
        else:
            lds = self.classes[self._lead].native.lds_bytes_per_agent()
            self._lead_on_main = lds > 0 and 163840 // lds > 4
        #: coordinated rounds launch only the agents still active (mpcx_active_map +
        #: mpcx_batch_solve_mapped): each class's solve is ``bound`` workgroups over the compacted
        #: agent map, the bound being the class's active count at the last stopping check (the
        #: active set only shrinks within a round); MPCX_FLEET_MAP=0 launches every agent
        self.map_launch = os.environ.get("MPCX_FLEET_MAP", "1") != "0" and hasattr(self.ops, "active_map")
        #: a class's per-iteration row moves (means / multipliers / penalty into p, locals out of w)
        #: as one scatter and one gather launch (C ABI v12); MPCX_FLEET_FUSED=0: one launch per move
        self.fused_moves = os.environ.get("MPCX_FLEET_FUSED", "1") != "0" and hasattr(self.ops, "scatter_plan")
        #: the per-iteration bookkeeping of all classes in one launch each (stats count, block
        #: expansion; C ABI v15); MPCX_FLEET_BOOK=0: one launch per class (A/B)
        self.fused_book = self.fused_moves and os.environ.get("MPCX_FLEET_BOOK", "1") != "0"
        self._stats_plans = {}  # freeze-mask mode -> prepared mpcx_stats_count_multi launch
        self._expand_key, self._expand_plan = None, None
        self._prepare_moves()
        self._mapped = False
        for c in self.classes:
            c.MAP = t.zeros(c.n, dtype=i32, device=dev)
            c.bound = c.n
        #: page-locked host twins of the buffers set_inputs / solutions move (see _pinned)
        self._host = {}
        self._host_ev = t.cuda.Event() if dev.type == "cuda" else None

    def set_inputs(self, class_name: str, p: np.ndarray, lbw: Optional[np.ndarray] = None,
                   ubw: Optional[np.ndarray] = None):
        """New measurements/forecasts for the next control step (host -> HBM);
        reference-layout arrays (lifted classes need all three)."""
        c = next(c for c in self.classes if c.name == class_name)
        p, lbw, ubw = c.to_kernel(p, lbw, ubw)
        for dst, src in ((c.P, p), (c.LB, lbw), (c.UB, ubw)):
            if src is not None:
                self._upload(dst, src)

    def _pinned(self, dev_t):
        """The page-locked host twin of a device buffer (made once): the fleet's host <-> device
        moves go through it.  A copy from pageable memory makes the HIP runtime lock the pages
        for the transfer and release them after it -- on a fresh numpy array every control step
        -- and the GPU work after such a step started 14-27 ms late in some processes (the C2
        leg's slow mode, r05/s20-s23)."""
        key = dev_t.data_ptr()
        buf = self._host.get(key)
        if buf is None or buf.shape != dev_t.shape:
            buf = self.torch.empty(dev_t.shape, dtype=dev_t.dtype, pin_memory=True)
            self._host[key] = buf
        return buf

    def _upload(self, dst, src):
        if self.device.type != "cuda":
            dst.copy_(self.torch.as_tensor(src))
            return
        h = self._pinned(dst)
        self._host_ev.synchronize()  # the previous upload out of this buffer is done
        np.copyto(h.numpy(), np.asarray(src, dtype=np.float64).reshape(h.shape))
        dst.copy_(h, non_blocking=True)
        self._host_ev.record()

    def _download(self, src) -> np.ndarray:
        if self.device.type != "cuda":
            return src.cpu().numpy()
        h = self._pinned(src)
        self._host_ev.synchronize()
        h.copy_(src, non_blocking=True)
        self.torch.cuda.current_stream(self.device).synchronize()
        return h.numpy().copy()

    def _sync(self):
        if self.device.type == "cuda":
            self.torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ steps
    def _set_blocks(self, rho_b: np.ndarray, active_b: Optional[np.ndarray]):
        """Upload the per-block penalties and (coordinated runs) the freeze masks -- only when
        they changed (most iterations change neither; each upload is a host round trip)."""
        t = self.torch
        key = (np.asarray(rho_b, float).tobytes(), None if active_b is None else np.asarray(active_b, bool).tobytes())
        if key == self._blk_key:
            return
        self._blk_key = key
        self.RHO_B.copy_(t.as_tensor(np.asarray(rho_b, float).reshape(-1, 1)))
        if self.G:
            self.RHO_G.copy_(t.as_tensor(np.asarray(rho_b, float)[self.block_of_group]))
        act = np.ones(self.n_blocks, bool) if active_b is None else np.asarray(active_b, bool)
        if self.G:
            self.ACTIVE_G.copy_(t.as_tensor(act[self.block_of_group].astype(np.int32)))
        masked = active_b is not None and not act.all()
        for ci, c in enumerate(self.classes):
            a = act[self.agent_blocks[ci]]
            if self._part is not None:
                a = a & self._part[ci]
                masked = masked or not self._part[ci].all()
            c.ACTIVE.copy_(t.as_tensor(a.astype(np.int32)))
        self._masked = masked

    def _scatter_moves(self, c):
        """Every row move into a class's p per iteration: each coupling slot's mean (or exchange
        diff) and multiplier columns, and the block's penalty."""
        T, moves = self.T, []
        for si, s in enumerate(c.slots):
            d = c.dev_slots[si]
            if s.kind == CONSENSUS:
                moves += [(T, self.MEAN, d["groups"], d["mean_cols"]), (T, self.LAMR, d["rows"], d["mult_cols"])]
            else:
                moves += [(T, self.DIFF, d["rows"], d["mean_cols"]), (T, self.GMULT, d["groups"], d["mult_cols"])]
        moves.append((1, self.RHO_B, c.BLOCK, c.RHO_COL))
        return moves

    def _gather_moves(self, c):
        """Each slot's local trajectory out of w; agents not participating keep their local
        (their rows map to the scratch row)."""
        part = getattr(self, "_part", None)
        return [(d["w_cols"], self.X, d["rows_part"] if part is not None else d["rows"]) for d in c.dev_slots]

    def _prepare_moves(self):
        """The fused moves of every class, prepared once (the buffers never move; the gathers
        again whenever the participation masks change): the iteration then issues each as one
        launch without building anything on the host -- a per-iteration list of moves was enough
        Python allocation to make the interpreter's collector show in the C2 leg."""
        if not getattr(self, "fused_moves", False):
            return
        for c in self.classes:
            c.scatter_plan = self.ops.scatter_plan(self._scatter_moves(c), c.P)
            g = self._gather_moves(c)
            c.gather_plan = self.ops.gather_plan(self.T, c.W, g) if g else None

    def _solve_all(self, rho: float):
        """Inject mean/diff, multipliers and the block's rho into every agent's p; solve
        (agents of frozen blocks are skipped); gather locals.

        The classes' solves are independent within an iteration (each agent reads the means and
        multipliers of the previous one), so with several classes each runs on a HIP stream of
        its own (``concurrent_classes``): a class's launch fills the CUs the other's leaves idle
        (its last, partial generation of agents), instead of starting after it."""
        ops, T, t = self.ops, self.T, self.torch
        streams = self._class_streams if self.concurrent_classes else None
        if streams:
            main = t.cuda.current_stream(self.device)
            self._ev_solve.record(main)
        lead = self._lead
        for ci in self._class_order:
            c = self.classes[ci]
            own = streams[ci] if streams and not (self._lead_on_main and ci == lead) else None
            with (t.cuda.stream(own) if own is not None else contextlib.nullcontext()):
                if own is not None:
                    # the other classes start once the lead class's solve is next in its queue: its
                    # workgroups claim the CUs first and the smaller classes fill what they leave
                    # (a class that needs a whole generation of the LDS, the C5 zones, split into two
                    # when the others' workgroups were dispatched beside it: r05/s14)
                    own.wait_event(self._ev_solve if ci == lead or lead is None else self._ev_lead)
                if self.fused_moves:  # every move of the class in one launch (C ABI v12), prepared
                    ops.run_plan(c.scatter_plan)
                else:
                    for T_, src, rows, cols in self._scatter_moves(c):
                        ops.scatter_rows(T_, src, rows, c.P, cols)
                if self._mapped:  # only the agents still active, compacted (mpcx_active_map)
                    ops.active_map(c.n, c.ACTIVE, c.MAP, self._map_counts[ci:ci + 1])
                if streams and ci == lead:
                    self._ev_lead.record(own if own is not None else main)
                if self._mapped:
                    ops.solve(c, c.ACTIVE, c.MAP, c.bound)
                else:
                    ops.solve(c, c.ACTIVE if self._masked else None)
                if self.fused_moves:
                    if c.gather_plan is not None:
                        ops.run_plan(c.gather_plan)
                else:
                    for cols, dst, rows in self._gather_moves(c):
                        ops.gather_rows(T, c.W, cols, dst, rows)
        if streams:
            for ci, st_ in enumerate(streams):
                if not (self._lead_on_main and ci == lead):
                    main.wait_stream(st_)
        if self.solve_trace is not None:
            for c in self.classes:
                words = c.ST.view(t.int32).view(c.n, STATS_BYTES // 4)
                self.solve_trace.append((c.name, words[:, _ITER_WORD:_STATUS_WORD + 1].clone()))
        # converged solves and restoration calls: every class in one launch (mpcx_stats_count_multi,
        # C ABI v15; the plan per freeze-mask mode), else one launch per class
        if self.fused_book and hasattr(ops, "stats_plan"):
            plan = self._stats_plans.get(self._masked)
            if plan is None:
                plan = self._stats_plans[self._masked] = ops.stats_plan(
                    [(c.n, c.ST, c.ACTIVE if self._masked else None) for c in self.classes], self._counts)
            ops.run_plan(plan)
        else:
            for c in self.classes:
                ops.stats_count(c.n, c.ST, c.ACTIVE if self._masked else None, self._counts)

    def _update_means(self, rho: float, apply_multipliers: bool, per_block: bool = False,
                      keep_control: bool = False):
        """Mean (+ exchange diffs) from the current locals; with ``apply_multipliers``
        also the multiplier update.  Returns the residual totals [n_blocks][8] (device).
        ``per_block``: per-group penalties and freeze masks of the coordinated run.  With
        several ranks every call is the iteration's one all-reduce (every rank calls it the
        same number of times: the ranks iterate in lockstep).  ``keep_control``: the control
        double holds this rank's count of active blocks (written by the stopping test of the
        coordinated loop) and is summed with the moments; otherwise it is zeroed with them, so
        a reduce outside that loop never sums a stale count (it would grow by a factor of the
        world size per call)."""
        ops, T, G, nb = self.ops, self.T, self.G, self.n_blocks
        if G == 0 and self.world == 1:
            return None
        rho_g = self.RHO_G if per_block else None
        act_g = self.ACTIVE_G if per_block and self._masked else None
        blk = self.BLOCK_G if nb > 1 else None
        # the moments buffer, and the control double unless the stopping test just wrote it
        (self.MOM if keep_control else self.MOMBUF).zero_()
        totals = self.MOM[self.totals_off:self.totals_off + ADMM_TOTALS * nb]
        exch = self.EXCH if self.exchange_flags.any() else None
        gm = self.GMULT if exch is not None else None
        if G:
            ops.moments(G, self.n_global, nb, T, self.GSTART, self.max_rows, self.X, self.LAMR, self.MEAN,
                        self.MOM, row_on=self.ROW_ON)
            ops.finalize(self.n_global, G, self.n_global, nb, T, self.MOM, exch, gm, rho, rho_g, act_g, blk,
                         self.MEAN, self.DMEAN, totals)
        if self.world > 1:  # the one collective, issued by the library (mpcx_admm_allreduce)
            self.collective.allreduce(self.reduce_len)
            self.n_collectives += 1
        if G == 0:
            return None
        if self.n_global:  # the groups spanning ranks, after their moments were summed
            ops.finalize(0, self.n_global, self.n_global, nb, T, self.MOM, exch, gm, rho, rho_g, act_g, blk,
                         self.MEAN, self.DMEAN, totals)
        # consensus rows of exchange groups are never read; exchange rows of consensus groups neither
        # (so a fleet of one kind launches only its own update)
        if apply_multipliers and not self.exchange_flags.all():
            ops.consensus_multipliers(G, T, self.GSTART, self.max_rows, self.X, self.MEAN, rho, rho_g, act_g,
                                      self.LAMR, row_on=self.ROW_ON)
        if exch is not None:
            ops.exchange_update(G, T, self.GSTART, self.max_rows, self.X, self.MEAN, self.DIFF, self.GMULT,
                                apply_multipliers, rho, rho_g, act_g, row_on=self.ROW_ON)
        return totals.view(nb, ADMM_TOTALS)

    def _shift_all(self, shift: int):
        """``shift_values_by_one`` of every variable (`admm_datatypes.py:275-282`, `326-331`):
        consensus means and multipliers; exchange multipliers and diffs — the mean of an
        exchange alias is NOT shifted."""
        ops, T = self.ops, self.T
        if self.G:
            # the exchange aliases' rows, a device index built once: a mask built from the host
            # flags here was a pageable host-to-device copy and two synchronisations per round,
            # which took 14-27 ms in some processes (r05/s20) against a 30 ms round
            if getattr(self, "_ex_rows", None) is None:
                self._ex_rows = self.torch.as_tensor(np.flatnonzero(np.asarray(self.exchange_flags)[:self.G]),
                                                     dtype=self.torch.int64, device=self.device)
            keep = self.MEAN.index_select(0, self._ex_rows) if self._ex_rows.numel() else None
            ops.shift(T, shift, self.MEAN)
            if keep is not None:
                self.MEAN.index_copy_(0, self._ex_rows, keep)
        ops.shift(T, shift, self.LAMR)
        ops.shift(T, shift, self.DIFF)
        ops.shift(T, shift, self.GMULT)

    # ------------------------------------------------------------------ algorithms
    def set_participation(self, participating: Optional[Dict[str, Sequence[bool]]] = None):
        """The agents taking part in the next rounds -- the reference coordinator's agents with
        status ``ready`` (`admm_coordinator.py:323-353`, `_agents_with_status`): only they are
        solved, enter the means, get their multipliers updated and count in the residuals
        (``sources=active_agents``, `admm_datatypes.py:171-331`); the others keep their local
        trajectories and multipliers (which are still shifted between control steps).
        ``participating`` maps class names to a bool per agent (missing classes: all
        agents); None: every agent."""
        t = self.torch
        self._blk_key = None
        if participating is None:
            self._part, self.ROW_ON = None, None
            for c in self.classes:
                c.PART = None
            self._prepare_moves()
            return
        part = []
        on = np.ones(self.X.shape[0], np.int32)
        for ci, c in enumerate(self.classes):
            m = np.ones(c.n, bool) if c.name not in participating else np.asarray(participating[c.name], bool)
            if m.shape != (c.n,):
                raise ValueError(f"{c.name}: participation mask of {m.shape}, {c.n} agents")
            part.append(m)
            for si, s in enumerate(c.slots):
                rows = np.asarray(self.slot_rows[(ci, si)])
                on[rows] = m.astype(np.int32)
                c.dev_slots[si]["rows_part"] = t.as_tensor(np.where(m, rows, self.X.shape[0] - 1).astype(np.int32),
                                                           device=self.device)
        self._part = part
        self._prepare_moves()  # the gathers read the new row maps
        for c, m in zip(self.classes, part):
            c.PART = t.as_tensor(m.astype(np.int32), device=self.device)
        self.ROW_ON = t.as_tensor(on, device=self.device)

    def register(self, class_name: str, agent: Optional[int]):
        """(Re-)registration of one agent (``ADMMCoordinator.register_agent``,
        `admm_coordinator.py:527-560`): its local trajectories restart from the configured
        initial value, its consensus multipliers from zero, and -- as the reference does --
        the multiplier of every exchange alias it joins is reset to zero; its backend starts
        cold (the NLP guess of the class's initial inputs).

        ``agent`` is the rank-local index of the agent, or None on the ranks that do not
        hold it.  With several ranks the call is collective (every rank calls it): an
        exchange alias whose participants span ranks keeps a replicated multiplier on each
        of them, so every rank resets the aliases the agent joins."""
        t = self.torch
        ci = next(i for i, c in enumerate(self.classes) if c.name == class_name)
        c = self.classes[ci]
        reset = []
        if agent is not None:
            for si, s in enumerate(c.slots):
                row = int(self.slot_rows[(ci, si)][agent])
                self.X[row] = float(s.initial[agent])
                self.LAMR[row] = 0.0
                self.DIFF[row] = 0.0
                if s.kind == EXCHANGE:
                    reset.append(s.aliases[agent])
            c.W[agent].copy_(t.as_tensor(c.w0[agent], device=self.device))
        if self.world > 1:
            gathered = [None] * self.world
            self.dist.all_gather_object(gathered, reset, group=self.group)
            reset = [al for lst in gathered for al in lst]
        gid = {al: i for i, al in enumerate(self.aliases)}
        for al in dict.fromkeys(reset):
            if al in gid:
                self.GMULT[gid[al]] = 0.0

    def run_coordinated(self, penalty_factor: float, admm_iter_max: int = 20, primal_tol: float = 1e-3,
                        dual_tol: float = 1e-3, use_relative_tolerances: bool = True, abs_tol: float = 1e-3,
                        rel_tol: float = 1e-3, penalty_change_threshold: float = -1.0,
                        penalty_change_factor: float = 2.0, check_every: int = 4) -> dict:
        """One control step of the coordinator (`admm_coordinator.py:259-321`), run by every
        block independently: its own residual test, penalty variation and iteration count;
        a converged block is frozen (no solves, no updates) while the others go on.

        The stopping test runs on the device (``mpcx_admm_block_stop``, one thread per block,
        after each iteration's residual totals): the block penalties, freeze masks, records and
        iteration counts stay in HBM, so an iteration issues launches only.  The host reads the
        number of blocks still active every ``check_every`` iterations and the records once,
        after the round; iterations run past the last block's stop before that check are no-ops
        (every agent and group frozen) and are not counted.  With several ranks the count
        travels in the control double of the iteration's one all-reduce (C ABI v10): after the
        reduce it is the count over all ranks after the PREVIOUS iteration, so every rank leaves
        the loop at the same iteration without a second collective.  Per-iteration wall times
        are device-clock stamps of the end of each iteration relative to the round's first stamp.

        Returns ``iterations`` (the last iteration any block ran), ``converged`` (all blocks),
        ``block_iterations`` / ``block_converged`` / ``block_records`` per block and
        ``records`` (block 0's history when there is one block, else the per-iteration
        norms over the blocks still running)."""
        t = self.torch
        ops, nb = self.ops, self.n_blocks
        dev, i32 = self.device, t.int32
        t0 = time.perf_counter()  # _performance_counter, set at the start of the round (:270)
        marks = [("entry", t0)] if _DEBUG else None
        rho0 = float(penalty_factor)
        n_it = max(int(admm_iter_max), 0)
        ACTIVE_B = t.ones(nb, dtype=i32, device=dev)
        ITERS_B = t.full((nb,), n_it, dtype=i32, device=dev)
        REC = t.zeros(max(n_it, 1) * nb * 4, dtype=t.float64, device=dev)
        # [n_active per iteration | each class's active-agent count of the last compaction]: what
        # a stopping check reads, in one copy
        CHK = t.zeros(n_it + 1 + len(self.classes), dtype=i32, device=dev)
        NACT = CHK[:n_it + 1]
        self._map_counts = CHK[n_it + 1:]
        self._mapped = self.map_launch
        for c in self.classes:
            c.bound = c.n
        CLOCK = t.zeros(n_it + 1, dtype=t.int64, device=dev)
        self.RHO_B.fill_(rho0)
        self._expand_blocks(ACTIVE_B)
        self._blk_key = None
        self._masked = True
        crit = (1 if use_relative_tolerances else 0, abs_tol, rel_tol, primal_tol, dual_tol,
                penalty_change_threshold, penalty_change_factor)
        coll0 = self.n_collectives
        if marks is not None:
            marks.append(("alloc", time.perf_counter()))
        self._update_means(rho0, apply_multipliers=False, per_block=True)
        if marks is not None:
            marks.append(("means", time.perf_counter()))
        shift = int(len(self.classes[0].coupling_grid) / self.classes[0].horizon)
        self._shift_all(shift)
        if marks is not None:
            marks.append(("shift", time.perf_counter()))
        self._counts.zero_()
        tot = self.MOM[self.totals_off:self.totals_off + ADMM_TOTALS * nb]
        multi = self.world > 1
        ctrl = self.CONTROL if multi else None
        # the round's first stamp (and, with several ranks, the starting count into the control)
        ops.block_stop(0, tot, crit, self.RHO_B, ACTIVE_B, ITERS_B, REC, NACT, CLOCK, ctrl)
        if marks is not None:
            self._sync()
            marks.append(("prologue", time.perf_counter()))
        ran = executed = 0
        every = max(int(check_every), 1)
        for it in range(1, n_it + 1):
            self._solve_all(rho0)
            # ranks iterate in lockstep (the loop exit below is agreed on), so every rank takes
            # part in every iteration's all-reduce; frozen groups' moments travel but are not used
            tot = self._update_means(rho0, apply_multipliers=True, per_block=True, keep_control=multi)
            executed = it
            if multi and it > 1 and (it - 1) % every == 0:
                left = float(self.CONTROL.item())  # the count over all ranks after iteration it - 1
                self._take_bounds(CHK)
                if left == 0.0:
                    break  # every block on every rank had stopped by iteration it - 1: this one was a no-op
            ops.block_stop(it, tot, crit, self.RHO_B, ACTIVE_B, ITERS_B, REC, NACT, CLOCK, ctrl)
            self._expand_blocks(ACTIVE_B)
            ran = it
            if not multi and (it % every == 0 or it == n_it):
                if self._take_bounds(CHK)[it] == 0:
                    break
        self._sync()
        if marks is not None:
            marks.append(("loop", time.perf_counter()))
        # the next round starts from full penalties and no freeze mask
        self._masked = False
        self._mapped = False
        self._blk_key = None
        wall = time.perf_counter() - t0
        iters = ITERS_B.cpu().numpy().astype(np.int64)
        conv_b = ACTIVE_B.cpu().numpy() == 0
        last = int(iters.max()) if nb else 0
        rec = REC.cpu().numpy().reshape(max(n_it, 1), nb, 4)[:ran]
        clk = CLOCK.cpu().numpy()
        hz = ops.clock_hz()
        block_records = _BlockRecords(nb)
        records = []
        for j in range(min(last, ran)):
            r = rec[j]
            a = r[:, 3] != 0
            now_t = float(clk[j + 1] - clk[0]) / hz
            block_records.append(r[:, 0], r[:, 1], r[:, 2], a, now_t)
            if nb == 1:
                continue
            records.append(IterationRecord(float(np.sqrt((r[a, 0] ** 2).sum())), float(np.sqrt((r[a, 1] ** 2).sum())),
                                           float(np.mean(r[a, 2])), wall_time=now_t))
        if nb == 1:
            records = block_records[0]
        self.history.extend(records)
        self.rounds += 1
        if marks is not None and self.device.type == "cuda":
            marks.append(("records", time.perf_counter()))
            print("[fleet] round " + " ".join(f"{n}={(t - t0) * 1e3:.2f}" for n, t in marks[1:]) + f" it={ran}",
                  file=sys.stderr, flush=True)
        return {"iterations": last, "converged": bool(conv_b.all()), "records": records, "wall_s": wall,
                "converged_solves": int(self._counts[0].item()), "block_iterations": iters,
                "block_converged": conv_b, "block_records": block_records, "block_is_global": self.block_is_global.copy(),
                "restorations": int(self._counts[1].item()), "loop_iterations": ran,
                "iterations_executed": executed, "collectives": self.n_collectives - coll0}

    def _take_bounds(self, chk) -> np.ndarray:
        """Read a stopping check's counters (one copy) and take each class's active-agent count
        of the last compaction as its launch size for the rest of the round."""
        h = chk.cpu().numpy()
        if self._mapped:
            for c, n in zip(self.classes, h[len(h) - len(self.classes):]):
                c.bound = int(n)
        if _DEBUG:  # diagnostics: the launch sizes a round takes
            print(f"[fleet] mapped={self._mapped} bounds={[c.bound for c in self.classes]} "
                  f"t={time.perf_counter():.4f}", file=sys.stderr, flush=True)
        return h

    def _expand_blocks(self, active_b):
        """Per-block penalties and freeze masks (device) to the groups and the agents (with the
        participation mask) -- what the solves, means and multiplier updates read."""
        ops = self.ops
        if self.fused_book and hasattr(ops, "expand_plan"):
            # the groups' and every class's expansion in one launch (mpcx_admm_block_expand_multi, C ABI
            # v15), the plan rebuilt when the round's block mask or a participation mask is new
            key = (active_b.data_ptr(),
                   tuple(None if getattr(c, "PART", None) is None else c.PART.data_ptr() for c in self.classes))
            if self._expand_key != key:
                entries = ([(self.BLOCK_G, None, self.ACTIVE_G, self.RHO_G)] if self.G else []) + \
                          [(c.BLOCK, getattr(c, "PART", None), c.ACTIVE, None) for c in self.classes]
                self._expand_plan = ops.expand_plan(entries, active_b, self.RHO_B)
                self._expand_key = key
            ops.run_plan(self._expand_plan)
            return
        if self.G:
            ops.block_expand(self.BLOCK_G, active_b, self.RHO_B, None, self.ACTIVE_G, self.RHO_G)
        for c in self.classes:
            ops.block_expand(c.BLOCK, active_b, None, getattr(c, "PART", None), c.ACTIVE, None)

    def save_stats(self, path, start_time: float, records: Sequence[IterationRecord], first_iteration: int = 0):
        """Append one round's residual history to the coordinator's ``solve_stats_file``
        (``ADMMCoordinator._save_stats``, `admm_coordinator.py:437-465`): index
        ``(start_time, iteration)``, columns primal_residual, dual_residual,
        penalty_parameter, wall_time."""
        import pandas as pd
        from pathlib import Path

        path = Path(path)
        header = not path.is_file()
        df = pd.DataFrame({"primal_residual": [r.primal_residual for r in records],
                           "dual_residual": [r.dual_residual for r in records],
                           "penalty_parameter": [r.penalty for r in records],
                           "wall_time": [r.wall_time for r in records]},
                          index=[(start_time, first_iteration + i) for i in range(len(records))])
        path.parent.mkdir(exist_ok=True, parents=True)
        df.to_csv(path_or_buf=path, header=header, mode="a")

    def run_local(self, penalty_factor: float, max_iterations: int, record_residuals: bool = True) -> dict:
        """One control step of decentralised ADMM (``LocalADMM.process``, `admm.py:873-937`)."""
        rho = float(penalty_factor)
        grid = self.classes[0].coupling_grid
        ts = self.classes[0].time_step
        shift = next(i for i, t in enumerate(grid) if t >= ts)
        self.ops.shift(self.T, shift, self.X)   # _shift_and_send_coupling_outputs
        self.ops.shift(self.T, shift, self.LAMR)  # _shift_multipliers
        self.ops.shift(self.T, shift, self.GMULT)
        self._set_blocks(np.full(self.n_blocks, rho), None)
        self._update_means(rho, apply_multipliers=False)  # _set_mean_coupling_values
        hist = self.torch.zeros((max(max_iterations, 1), ADMM_TOTALS), dtype=self.torch.float64,
                                device=self.device)
        t0 = time.perf_counter()
        self._counts.zero_()
        for it in range(max_iterations):
            self._solve_all(rho)
            tot = self._update_means(rho, apply_multipliers=True)
            if record_residuals and tot is not None:
                hist[it].copy_(tot.sum(0))
        h = hist.cpu().numpy()
        wall = time.perf_counter() - t0
        records = [IterationRecord(math.sqrt(max(r[0], 0.0)), math.sqrt(max(r[1], 0.0)), rho)
                   for r in h[:max_iterations]] if record_residuals else []
        self.history.extend(records)
        self.rounds += 1
        return {"iterations": max_iterations, "converged": None, "records": records, "wall_s": wall,
                "converged_solves": int(self._counts[0].item()),
                "restorations": int(self._counts[1].item())}

    # ------------------------------------------------------------------ outputs
    def solutions(self, class_name: str) -> np.ndarray:
        """Reference-layout NLP solution vectors [n, nw] of one class."""
        c = next(c for c in self.classes if c.name == class_name)
        return c.backend.problem.from_kernel(self._download(c.W), c.lbw_ref)

    def stats(self, class_name: str) -> list:
        from agentlib_mpc_amd.runtime.native import stats_to_dicts

        c = next(c for c in self.classes if c.name == class_name)
        return stats_to_dicts(c.ST.cpu().numpy().tobytes())

    def trajectories(self) -> Dict[str, np.ndarray]:
        """Mean trajectory per alias (``ConsensusVariable.mean_trajectory``)."""
        m = self.MEAN.cpu().numpy()
        return {al: m[i].copy() for i, al in enumerate(self.aliases)}

    def locals_of(self, class_name: str, slot: str) -> np.ndarray:
        ci = next(i for i, c in enumerate(self.classes) if c.name == class_name)
        si = next(i for i, s in enumerate(self.classes[ci].slots) if s.name == slot)
        return self.X.cpu().numpy()[self.slot_rows[(ci, si)]]

    def multipliers_of(self, class_name: str, slot: str) -> np.ndarray:
        ci = next(i for i, c in enumerate(self.classes) if c.name == class_name)
        si = next(i for i, s in enumerate(self.classes[ci].slots) if s.name == slot)
        s = self.classes[ci].slots[si]
        if s.kind == CONSENSUS:
            return self.LAMR.cpu().numpy()[self.slot_rows[(ci, si)]]
        return self.GMULT.cpu().numpy()[self.slot_groups[(ci, si)]]
