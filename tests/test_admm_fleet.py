"""Fleet ADMM driver host logic on CPU (test-side device ops, oracle IPM solves)
against the oracle's loop restatements of the reference
(`oracle/admm.py`: ``coordinated_round`` = ADMMCoordinator._fast_process,
``local_round`` = LocalADMM.process), and the partitioned (world_size 2, gloo)
driver against the single-process one.

Tolerances (north star, fp64): consensus / residual histories rel 1e-5.
"""

import os
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.admm.fleet import ADMMFleet
from agentlib_mpc_amd.runtime import collective, native
from oracle import admm as oadmm
from oracle import nlps
from tests.admm_cases import C2Oracle, C4Oracle, participation_rounds
from tests.cpu_admm_ops import CpuADMMOps

RTOL = 1e-5


def _c4_ops(N):
    return CpuADMMOps({"room": nlps.exchange_room(N=N), "supply": nlps.exchange_supply(N=N)})


def _c2_ops(N):
    return CpuADMMOps({"room": nlps.admm_room(N=N), "ahu": nlps.admm_ahu(N=N)})


def test_fleet_groups_and_rows():
    classes = bm.c2_fleet_classes(n_blocks=2, N=2)
    fl = ADMMFleet(classes, device="cpu", ops=_c2_ops(2))
    assert fl.G == 8 and fl.R == 16 and fl.max_rows == 2
    assert list(fl.gstart) == list(range(0, 17, 2))
    # every alias: one room row then the air handler row
    for g, al in enumerate(fl.aliases):
        i, b = int(al[4]) - 1, int(al.split("_b")[1])
        assert fl.slot_rows[(0, 0)][4 * b + i] == 2 * g
        assert fl.slot_rows[(1, i)][b] == 2 * g + 1


def test_local_exchange_round_matches_oracle():
    N, iters = 4, 3
    fl = ADMMFleet(bm.c4_fleet_classes(n_rooms=2, n_supply=1, N=N), device="cpu", ops=_c4_ops(N))
    out = fl.run_local(penalty_factor=1e4, max_iterations=iters)
    orc = C4Oracle(N, bm.C4_ROOMS[:2])
    shift = 1  # first multiple-shooting grid point >= ts
    state, hist = oadmm.local_round(orc.participation, orc.initial, orc, 1e4, shift, iters, T=N)
    np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], hist[-1]["mDot_coupling"],
                               rtol=RTOL, atol=1e-9)
    np.testing.assert_allclose(fl.locals_of("room", "mDot_out")[1], state["local"][("room1", "mDot_coupling")],
                               rtol=RTOL, atol=1e-9)
    np.testing.assert_allclose(fl.multipliers_of("supply", "mDot_out")[0],
                               state["mult"][("supply0", "mDot_coupling")], rtol=RTOL, atol=1e-6)
    assert out["converged_solves"] == 3 * iters


def test_coordinated_consensus_round_matches_oracle():
    N, iters = 2, 3
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N), device="cpu", ops=_c2_ops(N))
    out = fl.run_coordinated(0.4, admm_iter_max=iters, use_relative_tolerances=False, primal_tol=0.002,
                             dual_tol=0.1)
    orc = C2Oracle(N, bm.C2_ROOMS)
    state, hist, it, conv = oadmm.coordinated_round(
        orc.participation, orc.initial, orc, 0.4, N, iters, primal_tol=0.002, dual_tol=0.1,
        use_relative_tolerances=False, T=3 * N)
    assert out["iterations"] == it and out["converged"] == conv
    got = np.array([[r.primal_residual, r.dual_residual] for r in out["records"]])
    np.testing.assert_allclose(got, np.array(hist)[:, :2], rtol=RTOL, atol=1e-10)
    for i in range(4):
        al = f"mDot{i + 1}_coupling_b0"
        np.testing.assert_allclose(fl.trajectories()[al], state["vars"][al].mean, rtol=RTOL, atol=1e-10)


def test_coordinated_closed_loop_rounds_match_oracle():
    """Two control steps of the coordinator with new room measurements between
    them: mean update from the last round's locals, shift of means
    and multipliers by one interval (`admm_coordinator.py:278-279`,
    `admm_datatypes.py:275-331`), warm-started local solves, varying penalty
    (`admm_coordinator.py:467-479`) — residual histories and means per round."""
    N, iters = 2, 3
    classes = bm.c2_fleet_classes(n_blocks=1, N=N)
    fl = ADMMFleet(classes, device="cpu", ops=_c2_ops(N))
    orc = C2Oracle(N, bm.C2_ROOMS)
    kw = dict(admm_iter_max=iters, use_relative_tolerances=False, primal_tol=1e-9, dual_tol=1e-9,
              penalty_change_threshold=1.5, penalty_change_factor=1.3)
    be_r, cv_r = bm.admm_room(N=N)
    state = None
    for step in range(2):
        rooms = [(d, T0 - 0.7 * step) for d, T0 in bm.C2_ROOMS]
        if step:
            p, lbw, ubw, _ = bm._class_inputs(be_r, cv_r, {"T": [r[1] for r in rooms],
                                                           "d": [r[0] for r in rooms]}, 4)
            fl.set_inputs("room", p, lbw, ubw)
            orc.rooms = rooms
        out = fl.run_coordinated(0.4, **kw)
        state, hist, it, conv = oadmm.coordinated_round(orc.participation, orc.initial, orc, 0.4, N,
                                                        T=3 * N, state=state, **kw)
        assert out["iterations"] == it
        got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(hist), rtol=RTOL, atol=1e-10)
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b0"
            np.testing.assert_allclose(fl.trajectories()[al], state["vars"][al].mean, rtol=RTOL, atol=1e-10)


def test_coordinated_exchange_round_matches_oracle():
    """Coordinator-driven exchange ADMM (examples/exchange_admm with the coordinator):
    the exchange alias's mean is not shifted between rounds — only its multiplier and
    the diffs are (`ExchangeVariable.shift_values_by_one`, `admm_datatypes.py:326-331`) —
    so the first dual residual is taken against the unshifted mean."""
    N, iters = 3, 3
    fl = ADMMFleet(bm.c4_fleet_classes(n_rooms=2, n_supply=1, N=N), device="cpu", ops=_c4_ops(N))
    orc = C4Oracle(N, bm.C4_ROOMS[:2])
    kw = dict(admm_iter_max=iters, use_relative_tolerances=False, primal_tol=1e-12, dual_tol=1e-12)
    state = None
    for step in range(2):
        out = fl.run_coordinated(1e4, **kw)
        state, hist, it, conv = oadmm.coordinated_round(orc.participation, orc.initial, orc, 1e4, N, T=N,
                                                        state=state, **kw)
        assert out["iterations"] == it
        got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(hist), rtol=RTOL, atol=1e-10)
        np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], state["vars"]["mDot_coupling"].mean,
                                   rtol=RTOL, atol=1e-10)
        np.testing.assert_allclose(fl.multipliers_of("supply", "mDot_out")[0], state["vars"]["mDot_coupling"].mult,
                                   rtol=RTOL, atol=1e-6)


def test_blocks_run_like_their_own_coordinators():
    """Two independent 4-room blocks in one fleet: per-block stopping test and penalty
    variation; each block's history equals a single-block run of that block."""
    N = 2
    kw = dict(admm_iter_max=4, use_relative_tolerances=False, primal_tol=1e-3, dual_tol=5e-3,
              penalty_change_threshold=1.5, penalty_change_factor=1.3)
    two = ADMMFleet(bm.c2_fleet_classes(n_blocks=2, N=N, seed=3), device="cpu", ops=_c2_ops(N))
    assert two.n_blocks == 2 and [two.block_index(f"mDot1_coupling_b{b}") for b in (0, 1)] == [0, 1]
    out = two.run_coordinated(0.4, **kw)
    for b in (0, 1):
        one = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N, seed=3, block_offset=b), device="cpu",
                        ops=_c2_ops(N))
        o1 = one.run_coordinated(0.4, **kw)
        assert out["block_iterations"][b] == o1["iterations"]
        assert bool(out["block_converged"][b]) == o1["converged"]
        got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["block_records"][b]])
        want = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in o1["records"]])
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12)
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b{b}"
            np.testing.assert_allclose(two.trajectories()[al], one.trajectories()[al], rtol=1e-9, atol=1e-12)


def test_local_exchange_closed_loop_rounds_match_oracle():
    """Three LocalADMM control steps (shift of own trajectory and multipliers,
    `admm.py:873-937`) with new room measurements between them."""
    N, iters = 4, 2
    fl = ADMMFleet(bm.c4_fleet_classes(n_rooms=2, n_supply=1, N=N), device="cpu", ops=_c4_ops(N))
    orc = C4Oracle(N, bm.C4_ROOMS[:2])
    be_r, cv_r = bm.exchange_room(N=N)
    state = None
    for step in range(3):
        rooms = [(d, T0 + 0.5 * step) for d, T0 in bm.C4_ROOMS[:2]]
        if step:
            p, lbw, ubw, _ = bm._class_inputs(be_r, cv_r, {"T": [r[1] for r in rooms],
                                                           "d": [r[0] for r in rooms]}, 2)
            fl.set_inputs("room", p, lbw, ubw)
            orc.rooms = rooms
        fl.run_local(penalty_factor=1e4, max_iterations=iters)
        state, hist = oadmm.local_round(orc.participation, orc.initial, orc, 1e4, 1, iters, T=N, state=state)
        np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], hist[-1]["mDot_coupling"],
                                   rtol=RTOL, atol=1e-9)
        np.testing.assert_allclose(fl.multipliers_of("supply", "mDot_out")[0],
                                   state["mult"][("supply0", "mDot_coupling")], rtol=RTOL, atol=1e-6)


def test_relative_tolerance_totals_match_oracle():
    """The moment identities behind the single all-reduce reproduce the
    reference's relative stopping quantities (admm_coordinator.py:405-419)."""
    N, iters = 2, 2
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N), device="cpu", ops=_c2_ops(N))
    out = fl.run_coordinated(0.4, admm_iter_max=iters, use_relative_tolerances=True, abs_tol=1e-12,
                             rel_tol=1e-12, penalty_change_threshold=1.5)
    orc = C2Oracle(N, bm.C2_ROOMS)
    _, hist, it, _ = oadmm.coordinated_round(orc.participation, orc.initial, orc, 0.4, N, iters,
                                             use_relative_tolerances=True, abs_tol=1e-12, rel_tol=1e-12,
                                             penalty_change_threshold=1.5, T=3 * N)
    got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
    np.testing.assert_allclose(got, np.array(hist), rtol=RTOL, atol=1e-10)


# ---------------------------------------------------------------------------
# world_size 2 (gloo): agents partitioned across ranks, one all-reduce per iteration
# ---------------------------------------------------------------------------

def _worker(rank, world, init_file, N, iters, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        full = bm.c4_fleet_classes(n_rooms=4, n_supply=1, N=N)
        room, supply = full
        # rank r keeps rooms [2r, 2r+2); rank 0 also holds the supply unit
        from agentlib_mpc_amd.admm.fleet import FleetClass

        lo, hi = (2 * rank, 2 * rank + 2) if world == 2 else (0, 4)
        sl = lambda a: a[lo:hi]  # noqa: E731
        mine = [FleetClass("room", room.backend, (sl(room.p0), sl(room.lbw), sl(room.ubw), sl(room.w0)),
                           aliases={"mDot_out": "mDot_coupling"}, initial={"mDot_out": 0.02})]
        if rank == 0:
            mine.append(supply)
        fl = ADMMFleet(mine, device="cpu", ops=_c4_ops(N), comm="default" if world > 1 else None)
        out = fl.run_local(penalty_factor=1e4, max_iterations=iters)
        np.savez(f"{out_file}.{rank}.npz", mean=fl.trajectories()["mDot_coupling"],
                 prim=np.array([r.primal_residual for r in out["records"]]),
                 locals=fl.locals_of("room", "mDot_out"))
    finally:
        dist.destroy_process_group()


def _run(world, N, iters, tmp):
    init = os.path.join(tmp, f"init{world}")
    out = os.path.join(tmp, f"out{world}")
    mp.spawn(_worker, args=(world, init, N, iters, out), nprocs=world, join=True)
    return [dict(np.load(f"{out}.{r}.npz")) for r in range(world)]


def test_partitioned_fleet_world2_matches_world1():
    N, iters = 3, 2
    with tempfile.TemporaryDirectory() as tmp:
        one = _run(1, N, iters, tmp)[0]
        two = _run(2, N, iters, tmp)
    for r in two:
        np.testing.assert_allclose(r["mean"], one["mean"], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(r["prim"], one["prim"], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(np.concatenate([two[0]["locals"], two[1]["locals"]]), one["locals"],
                               rtol=1e-10, atol=1e-12)


def test_local_exchange_fleet_with_c_oracle_solves():
    """The fleet driver on the CPU (numpy ADMM arithmetic + C IPM over the host-compiled
    generated models, oracle/cpu_fleet.py) against `oracle/admm.local_round` with the same
    local solver per agent (tests/admm_cases.CFleetOracle): 60 rooms + 4 supply units on one
    exchange alias -- the CPU rehearsal of the 1024-agent GPU case."""
    from oracle.cpu_fleet import CpuFleetOps
    from tests.admm_cases import CFleetOracle

    N, iters = 10, 3
    classes = bm.c4_fleet_classes(n_rooms=60, n_supply=4, N=N, seed=11)
    fl = ADMMFleet(classes, device="cpu", ops=CpuFleetOps(bm.TIGHT["ipopt"], threads=2))
    fl.run_local(penalty_factor=1e4, max_iterations=iters)
    orc = CFleetOracle(classes, bm.TIGHT["ipopt"])
    state, hist = oadmm.local_round(orc.participation, orc.initial, orc, 1e4, 1, iters, T=N)
    np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], hist[-1]["mDot_coupling"], rtol=1e-7, atol=1e-9)
    loc = fl.locals_of("room", "mDot_out")
    want = np.array([state["local"][(f"room#{i}", "mDot_coupling")] for i in range(60)])
    # entries at the mDot >= 0 bound are interior-point distances ~1e-7 that move with the
    # barrier path (summation order of the mean): absolute 1e-7
    np.testing.assert_allclose(loc, want, rtol=1e-7, atol=1e-7)


def test_participation_and_registration_rounds_match_oracle():
    """Coordinator participation semantics (`admm_coordinator.py:323-353`,
    `:527-560`): a round without room 1 (not ready) and a round after its re-registration,
    fleet driver vs the oracle's coordinator restatement with the same active sets."""
    N, iters = 2, 2
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N), device="cpu", ops=_c2_ops(N))
    orc = C2Oracle(N, bm.C2_ROOMS)
    prev = None
    for step, (out, state, hist, it) in enumerate(participation_rounds(fl, orc, N, iters)):
        assert out["iterations"] == it, step
        room1 = fl.locals_of("room", "mDot")[1].copy()
        if step == 1:   # not ready: its local trajectory is not re-solved
            np.testing.assert_array_equal(room1, prev)
        prev = room1
        got = np.array([[r.primal_residual, r.dual_residual] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(hist)[:, :2], rtol=RTOL, atol=1e-10, err_msg=f"step {step}")
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b0"
            np.testing.assert_allclose(fl.trajectories()[al], state["vars"][al].mean, rtol=RTOL, atol=1e-10)
            np.testing.assert_allclose(fl.multipliers_of("ahu", f"mDot_out_{i + 1}")[0],
                                       state["vars"][al].mult["ahu"], rtol=RTOL, atol=1e-8)
        np.testing.assert_allclose(fl.locals_of("room", "mDot")[1], state["vars"]["mDot2_coupling_b0"].local["room1"],
                                   rtol=RTOL, atol=1e-10)


def _part_worker(rank, world, init_file, N, out_file):
    """Two C2 blocks, one per rank (world 2) or both on one rank (world 1); the second
    control step runs without room 1 of block 1 (not ready)."""
    if world > 1:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        classes = bm.c2_fleet_classes(n_blocks=2 if world == 1 else 1, N=N, seed=7,
                                      block_offset=0 if world == 1 else rank)
        fl = ADMMFleet(classes, device="cpu", ops=_c2_ops(N), comm="default" if world > 1 else None)
        kw = dict(admm_iter_max=1, use_relative_tolerances=False, primal_tol=1e-9, dual_tol=1e-9)
        first = fl.run_coordinated(0.4, **kw)
        if world == 1:
            mask = [True] * 5 + [False] + [True] * 2     # rooms of block 1 are agents 4..7
        else:
            mask = [True, False, True, True] if rank == 1 else [True] * 4
        fl.set_participation({"room": mask})
        out = fl.run_coordinated(0.4, **kw)
        traj = fl.trajectories()
        # per-block histories: world 1 holds blocks 0 and 1, rank r of world 2 block r (its
        # only, rank-local block); the all-reduce carries nothing for rank-local blocks but the
        # control double (the count of blocks still active that agrees the loop exit)
        assert fl.n_global_blocks == 0 and fl.reduce_len == 1 or world == 1
        rec = {f"rec{b if world == 1 else rank}": np.array(
            [[r.primal_residual, r.dual_residual] for r in first["block_records"][b] + out["block_records"][b]])
            for b in range(fl.n_blocks)}
        np.savez(f"{out_file}.{rank}.npz", **rec, **{al: traj[al] for al in traj})
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_partitioned_participation_world2_matches_world1(tmp_path):
    """Participation on a partitioned fleet (gloo, world_size 2): the masked rows drop out
    of the rank-local moments and the active-row counts travel in the one all-reduce, so
    two ranks with one block each give the one-rank result."""
    N = 2
    init, out = str(tmp_path / "init"), str(tmp_path / "out")
    _part_worker(0, 1, init, N, out + "1")
    one = dict(np.load(f"{out}1.0.npz"))
    mp.spawn(_part_worker, args=(2, init, N, out + "2"), nprocs=2, join=True)
    two = [dict(np.load(f"{out}2.{r}.npz")) for r in range(2)]
    for r in two:
        for al, v in r.items():
            np.testing.assert_allclose(v, one[al], rtol=1e-9, atol=1e-12, err_msg=al)


def test_masked_round_converging_at_first_iteration_keeps_the_mask():
    """A participation mask stays applied across rounds even when a round stops at its
    first iteration (the block-upload cache is dropped with the mask at the end of every
    round): the agent that is not ready is never solved, its warm start is untouched and it
    does not count as a converged solve."""
    N = 2
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N), device="cpu", ops=_c2_ops(N))
    fl.set_participation({"room": [True, False, True, True]})
    room = fl.classes[0]
    w1 = room.W[1].clone()
    kw = dict(admm_iter_max=5, use_relative_tolerances=False, primal_tol=1e9, dual_tol=1e9)
    for _ in range(2):
        out = fl.run_coordinated(0.4, **kw)
        assert out["iterations"] == 1 and out["converged"]
        assert out["converged_solves"] == 4          # rooms 0, 2, 3 and the air handler
        assert bool((room.W[1] == w1).all())


def _reg_worker(rank, world, init_file, N, out_file):
    """C4 exchange fleet, rooms split over the ranks (rank 0 also holds the supply unit);
    room 3 re-registers between two coordinated rounds.  With two ranks the exchange alias
    spans both, so every rank must reset its copy of the alias's multiplier."""
    if world > 1:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        from agentlib_mpc_amd.admm.fleet import FleetClass

        room, supply = bm.c4_fleet_classes(n_rooms=4, n_supply=1, N=N)
        lo, hi = (2 * rank, 2 * rank + 2) if world == 2 else (0, 4)
        sl = lambda a: a[lo:hi]  # noqa: E731
        mine = [FleetClass("room", room.backend, (sl(room.p0), sl(room.lbw), sl(room.ubw), sl(room.w0)),
                           aliases={"mDot_out": "mDot_coupling"}, initial={"mDot_out": 0.02})]
        if rank == 0:
            mine.append(supply)
        fl = ADMMFleet(mine, device="cpu", ops=_c4_ops(N), comm="default" if world > 1 else None)
        kw = dict(admm_iter_max=2, use_relative_tolerances=False, primal_tol=1e-12, dual_tol=1e-12)
        first = fl.run_coordinated(1e4, **kw)
        if world == 1:
            fl.register("room", 3)
        else:
            fl.register("room", 1 if rank == 1 else None)
        gm_after_reg = fl.GMULT[fl.aliases.index("mDot_coupling")].numpy().copy()
        out = fl.run_coordinated(1e4, **kw)
        np.savez(f"{out_file}.{rank}.npz", gm_reg=gm_after_reg,
                 gm=fl.GMULT[fl.aliases.index("mDot_coupling")].numpy(),
                 mean=fl.trajectories()["mDot_coupling"],
                 rec=np.array([[r.primal_residual, r.dual_residual] for r in first["records"] + out["records"]]))
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_partitioned_registration_world2_matches_world1(tmp_path):
    """Registration on a partitioned fleet: the exchange multiplier of a
    rank-spanning alias is reset on every rank, so both ranks keep the one-rank values."""
    N = 3
    init, out = str(tmp_path / "init"), str(tmp_path / "out")
    _reg_worker(0, 1, init, N, out + "1")
    one = dict(np.load(f"{out}1.0.npz"))
    assert not one["gm_reg"].any()
    mp.spawn(_reg_worker, args=(2, init, N, out + "2"), nprocs=2, join=True)
    two = [dict(np.load(f"{out}2.{r}.npz")) for r in range(2)]
    for r in two:
        assert not r["gm_reg"].any()
        np.testing.assert_allclose(r["rec"], one["rec"], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(r["gm"], one["gm"], rtol=1e-10, atol=1e-9)
        np.testing.assert_allclose(r["mean"], one["mean"], rtol=1e-10, atol=1e-12)


def test_consensus_multipliers_of_an_alias_sum_to_zero():
    """`tests/test_admm.py:147-161` property on the coordinated C2 fleet: every consensus
    alias's multipliers sum to zero over its participants (each update adds
    rho * (x_i - mean), whose sum over the participants vanishes)."""
    N = 2
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N), device="cpu", ops=_c2_ops(N))
    fl.run_coordinated(0.4, admm_iter_max=3, use_relative_tolerances=False, primal_tol=1e-12, dual_tol=1e-12)
    lam = fl.LAMR.numpy()
    assert np.abs(lam).max() > 0
    for g in range(fl.G):
        rows = lam[fl.gstart[g]:fl.gstart[g + 1]]
        assert len(rows) == 2
        np.testing.assert_allclose(rows.sum(0), 0.0, atol=1e-12 * np.abs(lam).max())


def _mixed_worker(rank, world, init_file, out_file, tols=(1e-12, 1e-12), iter_max=2, check_every=4):
    """One coordinated fleet holding a C4 exchange alias that spans the ranks (one global
    block) and C2 consensus blocks that are rank-local: world 1 holds everything, rank r of
    world 2 its share of the C4 agents and C2 block r."""
    if world > 1:
        dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    try:
        c2 = bm.c2_fleet_classes(n_blocks=2 if world == 1 else 1, N=1, seed=7,
                                 block_offset=0 if world == 1 else rank)
        c4 = bm.c4_fleet_classes(n_rooms=4, n_supply=2, N=3, rank=rank, world=world)
        for c in c4:
            c.name = "x" + c.name
        ops = CpuADMMOps({"room": nlps.admm_room(N=1), "ahu": nlps.admm_ahu(N=1),
                          "xroom": nlps.exchange_room(N=3), "xsupply": nlps.exchange_supply(N=3)})
        fl = ADMMFleet(c2 + c4, device="cpu", ops=ops, comm="default" if world > 1 else None)
        assert fl.n_global_blocks == (1 if world > 1 else 0)
        if world > 1:   # the exchange group's moments + ONE block's totals, whatever the C2 count
            # the length the C ABI defines (ctypes call of mpcx_admm_reduce_count, no GPU) is
            # the layout the fleet fills: global moments first, then the spanning block's totals
            assert fl.reduce_len == native.admm_reduce_count(fl.n_global, 1, fl.T)
            assert fl.reduce_len == 1 + fl.n_global * fl.S + 8   # control + moments + one block's totals
        calls = []
        real = dist.all_reduce
        if world > 1:   # count every collective the round issues
            dist.all_reduce = lambda *a, **k: (calls.append(a[0].numel()), real(*a, **k))[1]
            # the collective goes through the C ABI (mpcx_admm_allreduce, v14): the library's own
            # count of the collectives it issued, its transport the registered function (gloo)
            lib0 = collective.calls()
            assert collective.kind() == native.COLLECTIVE_FN
        try:
            out = fl.run_coordinated(1.0, admm_iter_max=iter_max, use_relative_tolerances=False,
                                     primal_tol=tols[0], dual_tol=tols[1], check_every=check_every)
        finally:
            dist.all_reduce = real
        if world > 1:
            # ONE all-reduce per ADMM iteration executed (plus the round's initial mean update),
            # each of the same length: no second collective for the loop exit
            assert len(calls) == out["collectives"] == 1 + out["iterations_executed"], (calls, out)
            assert collective.calls() - lib0 == len(calls), (collective.calls() - lib0, calls)
            assert set(calls) == {fl.reduce_len}, calls
            assert out["iterations_executed"] - out["loop_iterations"] <= 1
        xb = fl.block_index("mDot_coupling")
        np.savez(f"{out_file}.{rank}.iters.npz", iters=out["block_iterations"][[xb] + c2b_of(fl, world, rank)])
        c2b = [fl.block_index(f"mDot1_coupling_b{b}") for b in ((0, 1) if world == 1 else (rank,))]
        rec = {"x": np.array([[r.primal_residual, r.dual_residual] for r in out["block_records"][xb]])}
        for b, blk in zip((0, 1) if world == 1 else (rank,), c2b):
            rec[f"b{b}"] = np.array([[r.primal_residual, r.dual_residual] for r in out["block_records"][blk]])
        traj = fl.trajectories()
        np.savez(f"{out_file}.{rank}.npz", **rec, **{f"t_{al}": v for al, v in traj.items()})
    finally:
        if world > 1:
            dist.destroy_process_group()


def c2b_of(fl, world, rank):
    return [fl.block_index(f"mDot1_coupling_b{b}") for b in ((0, 1) if world == 1 else (rank,))]


@pytest.mark.parametrize("tols,iter_max,want_iters,check_every", [
    ((1e-12, 1e-12), 2, None, 4),
    # the spanning exchange block meets its rule at iteration 2 (primal 0.041 < 0.05, dual 2e-5 <
    # 1e-3) while the C2 blocks keep going to the cap: the ranks go on in lockstep (one all-reduce
    # per iteration, the stopped spanning block's moments travel but are not used)
    ((0.05, 1e-3), 5, (2, 5), 4),
    # every block stops early (loose rule): the loop exit is read from the control double of the
    # iteration's all-reduce, one iteration late at most, and both ranks leave together
    ((10.0, 10.0), 8, (1, 1), 1),
])
def test_mixed_global_and_local_blocks_world2_matches_world1(tmp_path, tols, iter_max, want_iters, check_every):
    """Blocks spanning ranks and rank-local blocks in one coordinated fleet: the
    spanning block's totals travel in the one all-reduce, the local blocks' do not, and two
    ranks reproduce the one-rank histories block by block -- also once the spanning block has
    stopped.  Exactly one all-reduce per ADMM iteration (patched ``dist.all_reduce``): the count
    of blocks still active rides in its control double."""
    init, out = str(tmp_path / "init"), str(tmp_path / "out")
    _mixed_worker(0, 1, init, out + "1", tols, iter_max, check_every)
    one = dict(np.load(f"{out}1.0.npz"))
    if want_iters is not None:
        it1 = np.load(f"{out}1.0.iters.npz")["iters"]
        assert it1[0] == want_iters[0] and (it1[1:] == want_iters[1]).all(), it1
    mp.spawn(_mixed_worker, args=(2, init, out + "2", tols, iter_max, check_every), nprocs=2, join=True)
    for r in range(2):
        two = dict(np.load(f"{out}2.{r}.npz"))
        assert f"b{r}" in two
        for k, v in two.items():
            np.testing.assert_allclose(v, one[k], rtol=1e-9, atol=1e-12, err_msg=k)
        if want_iters is not None:
            it2 = np.load(f"{out}2.{r}.iters.npz")["iters"]
            assert it2[0] == want_iters[0] and (it2[1:] == want_iters[1]).all(), it2


def test_device_stopping_test_reproduces_the_c2_coordinator_fixture_on_cpu():
    """The coordinators' stopping test as the fleet runs it now -- on the device state
    (``mpcx_admm_block_stop`` restated in numpy, `oracle/cpu_fleet.py`), the host reading the
    active-block count every few iterations -- against the oracle coordinator's host loop
    (`tests/golden/c2_admm_N10.json`: examples/4_Room_ADMM_Coordinator at its settings, N=10,
    run to its stopping rule): same stopping iteration, residual and penalty history, means.
    Local solves: the C IPM restatement at the fixture's settings."""
    import json
    from oracle.cpu_fleet import CpuFleetOps

    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c2_admm_N10.json")))
    for check_every in (1, 4, 7):
        fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=gold["N"]), device="cpu",
                       ops=CpuFleetOps(gold["solver"], threads=2))
        out = fl.run_coordinated(gold["rho"], admm_iter_max=gold["admm_iter_max"], check_every=check_every,
                                 **gold["criterion"])
        assert out["iterations"] == gold["iterations"] and out["converged"] == gold["converged"]
        assert out["loop_iterations"] - out["iterations"] < check_every
        got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(gold["history"]), rtol=1e-5, atol=1e-9)
        traj = fl.trajectories()
        for al, mean in gold["means"].items():
            np.testing.assert_allclose(traj[al], mean, rtol=1e-5, atol=1e-9)


def test_closed_loop_plant_update_takes_the_predicted_state():
    """``benchmarks.advance_plant`` (the coordinated bench legs' closed loop): after a round,
    each room's next measurement is its predicted temperature one interval ahead, and the
    uploaded NLP inputs equal a fresh marshalling of the rooms at those measurements."""
    N = 2
    classes = bm.c2_fleet_classes(n_blocks=1, N=N)
    fl = ADMMFleet(classes, device="cpu", ops=_c2_ops(N))
    fl.run_coordinated(0.4, admm_iter_max=2, use_relative_tolerances=False, primal_tol=1e-9, dual_tol=1e-9)
    room = classes[0]
    ts = room.backend.config.discretization_options.time_step
    w = fl.solutions("room")
    want_T = bm.value_at(room.backend.problem, w, "T", ts)
    assert np.all(np.abs(want_T - np.array([t for _, t in bm.C2_ROOMS])) > 0)
    bm.advance_plant(fl, ts)
    cv, vals, _ = room.plant
    np.testing.assert_array_equal(vals["T"], want_T)
    p, lbw, ubw, _ = bm._class_inputs(room.backend, cv, {"T": want_T, "d": [d for d, _ in bm.C2_ROOMS]}, 4)
    kp, kl, ku = room.to_kernel(p, lbw, ubw)
    np.testing.assert_array_equal(room.P.numpy(), kp)
    np.testing.assert_array_equal(room.LB.numpy(), kl)
