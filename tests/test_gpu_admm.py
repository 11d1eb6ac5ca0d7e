"""GPU parity of the ADMM path: the HIP ADMM kernels (C ABI) against their
numpy restatement, and the fleet driver on the GPU against the oracle's loop
restatements of the reference (`oracle/admm.py`) with oracle IPM solves.

Tolerances: kernels 1e-12 (fp64 atomics reorder sums); trajectories and
residual histories rel 1e-5 (north star).
"""

import json
import os

import numpy as np
import pytest
import torch

from agentlib_mpc_amd import benchmarks as bm
from agentlib_mpc_amd.admm.fleet import ADMMFleet
from agentlib_mpc_amd.admm.ops import NativeADMMOps
from oracle import admm as oadmm
from tests.admm_cases import C2Oracle, C4Oracle, CFleetOracle, participation_rounds
from tests.cpu_admm_ops import CpuADMMOps

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _pair(a):
    return torch.as_tensor(a).cuda(), torch.as_tensor(np.array(a, copy=True))


@pytest.mark.parametrize("T,sizes,n_global,n_blocks", [(10, [5, 1, 300, 2], 0, 1), (30, [2] * 7, 3, 3),
                                                        (300, [3, 600], 1, 1), (24, [3, 3, 3, 1, 5, 2], 2, 4)])
def test_admm_kernels_match_restatement(T, sizes, n_global, n_blocks):
    """Every ADMM kernel (moments, finalize with per-block totals, per-group penalties and
    a freeze mask, multiplier/diff updates, shift, row moves) against the numpy
    restatement of the same interface (tests/cpu_admm_ops.py)."""
    rng = np.random.default_rng(T)
    G = len(sizes)
    gstart = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    R = int(gstart[-1])
    X = rng.normal(0.02, 0.01, (R, T))
    LAM = rng.normal(0.0, 1.0, (R, T))
    MEAN = rng.normal(0.02, 0.01, (G, T))
    GM = rng.normal(0.0, 1.0, (G, T))
    EX = (np.arange(G) % 2).astype(np.int32)
    COLS = rng.permutation(T + 5)[:T].astype(np.int32)
    BLK = (np.arange(G) % n_blocks).astype(np.int32)
    RHO_G = rng.uniform(0.2, 2.0, G) if n_blocks > 1 else None
    ACT_G = (np.arange(G) % 3 != 1).astype(np.int32) if n_blocks > 1 else None
    ROW_ON = (rng.random(R) > 0.3).astype(np.int32) if n_blocks > 1 else None   # participation
    gpu, cpu = NativeADMMOps(), CpuADMMOps({})
    res = []
    for ops, mk in ((gpu, lambda a: _pair(a)[0]), (cpu, lambda a: _pair(a)[1])):
        gs, x, lam, mean, gm, ex = map(mk, (gstart, X, LAM, MEAN, GM, EX))
        blk = mk(BLK) if n_blocks > 1 else None
        rho_g = None if RHO_G is None else mk(RHO_G)
        act_g = None if ACT_G is None else mk(ACT_G)
        ron = None if ROW_ON is None else mk(ROW_ON)
        dmean = mk(np.zeros((G, T)))
        diff = mk(np.zeros((R, T)))
        mom = mk(np.zeros(ops.moments_size(G, n_blocks, T)))
        ops.moments(G, n_global, n_blocks, T, gs, max(sizes), x, lam, mean, mom, row_on=ron)
        off = n_global * (5 * T + 1)
        tot = mom[off:off + 8 * n_blocks]
        ops.finalize(n_global, G, n_global, n_blocks, T, mom, ex, gm, 0.7, rho_g, act_g, blk, mean, dmean, tot)
        ops.finalize(0, n_global, n_global, n_blocks, T, mom, ex, gm, 0.7, rho_g, act_g, blk, mean, dmean, tot)
        ops.consensus_multipliers(G, T, gs, max(sizes), x, mean, 0.7, rho_g, act_g, lam, row_on=ron)
        ops.exchange_update(G, T, gs, max(sizes), x, mean, diff, gm, True, 0.7, rho_g, act_g, row_on=ron)
        ops.shift(T, 3, lam)
        cols = mk(COLS)
        dst = mk(np.zeros((R, T + 5)))
        ops.scatter_rows(T, x, None, dst, cols)
        ops.fill_column(dst, 2, 1.5)
        back = mk(np.zeros((R, T)))
        ops.gather_rows(T, dst, cols, back, mk(np.arange(R, dtype=np.int32)[::-1].copy()))
        torch.cuda.synchronize()
        res.append([t.cpu().numpy() for t in (mom, mean, dmean, lam, diff, gm, dst, back)])
    for a, b in zip(*res):
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-13)


def test_gpu_local_exchange_fleet_matches_oracle():
    """examples/exchange_admm: 4 rooms + supply, N=10, ts=120, rho=1e4 (LocalADMM)."""
    N, iters = 10, 4
    fl = ADMMFleet(bm.c4_fleet_classes(n_rooms=4, n_supply=1, N=N))
    out = fl.run_local(penalty_factor=1e4, max_iterations=iters)
    assert out["converged_solves"] == 5 * iters
    orc = C4Oracle(N, bm.C4_ROOMS)
    state, hist = oadmm.local_round(orc.participation, orc.initial, orc, 1e4, 1, iters, T=N)
    np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], hist[-1]["mDot_coupling"],
                               rtol=RTOL, atol=1e-9)
    loc = fl.locals_of("room", "mDot_out")
    for i in range(4):
        np.testing.assert_allclose(loc[i], state["local"][(f"room{i}", "mDot_coupling")], rtol=RTOL, atol=1e-9)
    np.testing.assert_allclose(fl.multipliers_of("room", "mDot_out")[0],
                               state["mult"][("room0", "mDot_coupling")], rtol=RTOL, atol=1e-6)


def test_gpu_coordinated_fleet_matches_oracle():
    """examples/4_Room_ADMM_Coordinator: rho=0.4, N=10, ts=60, absolute criterion."""
    N, iters = 10, 3
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N))
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
        np.testing.assert_allclose(fl.multipliers_of("ahu", f"mDot_out_{i + 1}")[0],
                                   state["vars"][al].mult["ahu"], rtol=RTOL, atol=1e-8)


def test_gpu_coordinated_closed_loop_matches_oracle():
    """Two coordinator control steps on the GPU fleet with new room measurements
    between them: device-side mean update, shift of means/multipliers, warm-started
    batched solves and a varying penalty, against the oracle's round restatement."""
    N, iters = 10, 3
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N))
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
        state, hist, it, _ = oadmm.coordinated_round(orc.participation, orc.initial, orc, 0.4, N,
                                                     T=3 * N, state=state, **kw)
        assert out["iterations"] == it
        got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(hist), rtol=RTOL, atol=1e-10)
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b0"
            np.testing.assert_allclose(fl.trajectories()[al], state["vars"][al].mean, rtol=RTOL, atol=1e-10)


def test_gpu_participation_and_registration_match_oracle():
    """Coordinator participation on the GPU fleet (`admm_coordinator.py:323-353`,
    `:527-560`): room 1 not ready for one control step (masked out of the batched solve,
    the segmented means, multipliers and residual scalings), then re-registered with a
    cold start, against the oracle's coordinator restatement with the same active sets."""
    N, iters = 10, 3
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N))
    orc = C2Oracle(N, bm.C2_ROOMS)
    prev = None
    for step, (out, state, hist, it) in enumerate(participation_rounds(fl, orc, N, iters)):
        assert out["iterations"] == it, step
        got = np.array([[r.primal_residual, r.dual_residual] for r in out["records"]])
        np.testing.assert_allclose(got, np.array(hist)[:, :2], rtol=RTOL, atol=1e-10, err_msg=f"step {step}")
        room1 = fl.locals_of("room", "mDot")[1].copy()
        if step == 1:
            np.testing.assert_array_equal(room1, prev)
        prev = room1
        np.testing.assert_allclose(room1, state["vars"]["mDot2_coupling_b0"].local["room1"], rtol=RTOL, atol=1e-10)
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b0"
            np.testing.assert_allclose(fl.trajectories()[al], state["vars"][al].mean, rtol=RTOL, atol=1e-10)
            np.testing.assert_allclose(fl.multipliers_of("ahu", f"mDot_out_{i + 1}")[0],
                                       state["vars"][al].mult["ahu"], rtol=RTOL, atol=1e-8)


def _fleet_local_iterations(fl, n_iter):
    """Per ADMM iteration: every agent's local-solve IPM iteration count ({agent: n}) from the
    fleet's ``solve_trace`` (agent names as the oracle's C5 participation: zone0-2, ahu, cca)."""
    k = len(fl.classes)
    out = []
    for it in range(n_iter):
        row = {}
        for name, w in fl.solve_trace[it * k:(it + 1) * k]:
            w = w.cpu().numpy()
            for i in range(w.shape[0]):
                row[f"{name}{i}" if name == "zone" else name] = int(w[i, 0])
        out.append(row)
    return out


@pytest.mark.parametrize("N", [8, 24])
def test_gpu_three_zone_narx_fleet_matches_oracle_fixture(N):
    """examples/three_zone_datadriven_admm: 3 NARX zones + AHU + CCA (networks trained as
    the example trains them, `models/data/`), coordinated ADMM, rho=1, absolute criterion
    0.04/0.04, to the example's stopping rule (admm_iter_max 50), at N=8 and at the
    example's horizon N=24, against the oracle's round (`tests/golden/c5_admm_N{8,24}.json`,
    `tests/golden/make_admm_goldens.py`: hand-restated NLPs, oracle IPM and coordinator;
    both at tol 1e-8).

    The supply agents' costs are nearly non-smooth (sqrt(W^2 + 0.02) at objective scale ~1e6):
    their local solves end at the fp64 noise floor of tol 1e-8, so their IPM iteration counts
    differ between the two sides from the first iterations on while the solutions agree to
    ~1e-10 (N=8) / ~1e-6 (N=24) (scripts/c5_counts.py, profiles/r04/s3/c5_counts_n8.txt), and
    at some iteration one of them stops at a nearby point and the consensus paths part (a jump
    to 1e-2..1: iteration 44 at N=8, 40 at N=24 in r04; 12 at N=8, 40 at N=24 after the r05
    kernel's refined reciprocals, profiles/r05/s5/c5_fixtures.txt); which iteration depends on
    rounding, so it cannot be pinned tighter than a floor without pinning rounding itself.
    Evidence (r06, `scripts/c5_rounding_split.py`, CPU, oracle only): the ORACLE's own round with
    every local solve's start moved by a seeded relative 1e-12 parts from its fixture by the same
    rule at iteration 23, 10, 42, 12, 47, 43 or not within the 50 (seeds 1-8,
    profiles/r06/c5_rounding_split_n8*.txt; at N=24 profiles/r06/c5_rounding_split_n24.txt) -- the
    kernel's 12 is inside the oracle's own spread, and the first local solve whose IPM iteration
    count differs comes as early as iteration 2 while the residuals still agree to 1e-13.
    That iteration is found from the data -- the first whose residuals differ from the
    oracle's by more than 1e-3 relative -- and must not come before iteration 10 (N=8: the
    earliest oracle-vs-oracle split) / 30 (N=24).  The local
    IPM iteration counts (per-solve stats in the fixture) are reported, not compared: at tol
    1e-8 these solves stop at the rounding floor of the optimality error, so the counts differ
    between two correct runs (zones too at N=24) while the solutions agree.  After it: the
    stopping outcome, the residual levels of the last ten iterations (within 3x), and the final
    consensus means inside a band sized from the oracle's own sensitivity (how far its means
    still move after the divergence iteration)."""
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", f"c5_admm_N{N}.json")))
    opts = {"ipopt": {"tol": 1e-8, "max_iter": 500, "acceptable_iter": 0}}
    fl = ADMMFleet(bm.c5_fleet_classes(n_blocks=1, N=gold["N"], solver_options=opts))
    fl.solve_trace = []
    out = fl.run_coordinated(gold["rho"], admm_iter_max=gold.get("admm_iter_max", 50),
                             use_relative_tolerances=False, primal_tol=0.04, dual_tol=0.04, check_every=1)
    assert out["iterations"] == gold["iterations"] and out["converged"] == gold["converged"]
    got = np.array([[r.primal_residual, r.dual_residual] for r in out["records"]])
    want = np.array(gold["history"])[:, :2]
    rel = np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-3), axis=1)
    div = int(np.argmax(rel > 1e-3)) if np.any(rel > 1e-3) else len(want)
    print(f"C5 N={N}: residual histories part at iteration {div + 1} of {len(want)}")
    print("per-iteration relative residual difference:", np.array2string(rel, precision=2))
    # floors: N=24 parted at iteration 40 in r04 and r05 alike, N=8 at 44 then 12 (above)
    assert div >= {8: 10, 24: 30}.get(N, 10), (div, rel[:div + 1])
    kits = _fleet_local_iterations(fl, div)
    same = np.mean([kits[k][ag] == v[1] for k in range(div) for ag, v in gold["local_solves"][k].items()])
    print(f"local IPM iteration counts equal to the oracle's in {100 * same:.0f} % of the prefix's solves")
    traj = fl.trajectories()
    if div == len(want):
        for al, mean in gold["means"].items():
            np.testing.assert_allclose(traj[al], mean, rtol=RTOL, atol=1e-6)
        return
    tail = slice(max(div, len(want) - 10), len(want))
    for col in (0, 1):
        ratio = np.median(got[tail, col]) / np.median(want[tail, col])
        assert 1 / 3 < ratio < 3, (col, ratio)
    hist = gold["mean_history"]
    for al, mean in gold["means"].items():
        mean = np.asarray(mean)
        drift = max(np.max(np.abs(np.asarray(h[al]) - mean)) for h in hist[div:])
        dev = np.max(np.abs(traj[al] - mean))
        print(f"  {al}: |gpu - oracle| {dev:.3g}, oracle drift after iteration {div + 1}: {drift:.3g}")
        assert dev <= 3 * drift + 1e-6, (al, dev, drift)


def test_gpu_fleet_blocks_are_independent():
    """A scaled C2 fleet (many 4-room blocks, one launch per class) gives every
    block the trajectory a single-block run gives it."""
    N = 10
    big = ADMMFleet(bm.c2_fleet_classes(n_blocks=64, N=N, seed=5))
    big.run_coordinated(0.4, admm_iter_max=3, use_relative_tolerances=False, primal_tol=0.0, dual_tol=0.0)
    one = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N, seed=5, block_offset=37))
    one.run_coordinated(0.4, admm_iter_max=3, use_relative_tolerances=False, primal_tol=0.0, dual_tol=0.0)
    tb, to = big.trajectories(), one.trajectories()
    for i in range(4):
        al = f"mDot{i + 1}_coupling_b37"
        np.testing.assert_allclose(tb[al], to[al], rtol=1e-9, atol=1e-12)


def test_gpu_c2_coordinator_to_stopping_rule_matches_oracle_fixture():
    """examples/4_Room_ADMM_Coordinator at its coordinator settings (rho 0.4, absolute
    criterion 0.002 / 0.1, admm_iter_max 40, N=10) run to the stopping rule, against the
    oracle's round (`tests/golden/c2_admm_N10.json`, `tests/golden/make_admm_goldens.py`):
    same iteration count, residual and penalty history, final means."""
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "c2_admm_N10.json")))
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=gold["N"]))
    out = fl.run_coordinated(gold["rho"], admm_iter_max=gold["admm_iter_max"], **gold["criterion"])
    assert out["iterations"] == gold["iterations"] and out["converged"] == gold["converged"]
    got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
    np.testing.assert_allclose(got, np.array(gold["history"]), rtol=RTOL, atol=1e-10)
    traj = fl.trajectories()
    for al, mean in gold["means"].items():
        np.testing.assert_allclose(traj[al], mean, rtol=RTOL, atol=1e-10)


def test_gpu_stalled_c2_block_matches_oracle_fixture():
    """A block of the bench's scaled C2 fleet that does NOT converge within the coordinator's
    40 iterations (block 3 of seed 20261015 + 1, local solves at the reference's IPOPT
    settings as in the bench leg), against the oracle's round of the same block
    (`tests/golden/c2_admm_N10_b3.json`: hand-restated NLPs, oracle IPM at the same
    settings, oracle coordinator): same outcome, residual history, final means.  With the
    reference's acceptable-level local solves the primal residual levels off near 0.003,
    above the 0.002 tolerance; with tight local solves 99 % of the blocks converge
    (profiles/r03/s5/c2_conv.txt) -- the stall is the reference's settings, not the fleet."""
    path = os.path.join(os.path.dirname(__file__), "golden", "c2_admm_N10_b3.json")
    gold = json.load(open(path))
    b = gold["block"]
    fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=gold["N"], seed=gold["seed"], block_offset=b,
                                       solver_options={"ipopt": {}}))
    out = fl.run_coordinated(gold["rho"], admm_iter_max=gold["admm_iter_max"], **gold["criterion"])
    assert out["iterations"] == gold["iterations"] and out["converged"] == gold["converged"]
    assert not gold["converged"] and gold["iterations"] == gold["admm_iter_max"]
    got = np.array([[r.primal_residual, r.dual_residual, r.penalty] for r in out["records"]])
    want = np.array(gold["history"])
    rel = np.max(np.abs(got - want) / np.maximum(np.abs(want), 1e-4), axis=1)
    print("C2 block %d per-iteration relative residual difference:" % b, np.array2string(rel, precision=2))
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)
    traj = fl.trajectories()
    for al, mean in gold["means"].items():
        np.testing.assert_allclose(traj[al.replace("_b0", f"_b{b}")], mean, rtol=1e-6, atol=1e-9)


def test_gpu_every_block_stops_like_its_own_coordinator():
    """A 64-block C2 fleet (one launch per class and iteration): every block keeps its own
    stopping test and is frozen once converged, so each block ends at the iteration, with
    the residual history and means, of a single-block run of that block alone (one
    reference ADMMCoordinator, `admm_coordinator.py:284-309`)."""
    N, kw = 10, dict(admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
    big = ADMMFleet(bm.c2_fleet_classes(n_blocks=64, N=N, seed=5))
    assert big.n_blocks == 64
    out = big.run_coordinated(0.4, **kw)
    its = np.asarray(out["block_iterations"])
    assert out["converged"] and len(set(its.tolist())) > 1, its   # blocks stop at different iterations
    tb = big.trajectories()
    seed_block = {big.block_index(f"mDot1_coupling_b{b}"): b for b in range(64)}
    assert sorted(seed_block) == list(range(64))
    for k in sorted({big.block_index("mDot1_coupling_b0"), int(np.argmin(its)), int(np.argmax(its)),
                     big.block_index("mDot1_coupling_b37")}):
        b = seed_block[k]
        one = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N, seed=5, block_offset=b))
        o1 = one.run_coordinated(0.4, **kw)
        assert its[k] == o1["iterations"], (b, its[k], o1["iterations"])
        got = np.array([[r.primal_residual, r.dual_residual] for r in out["block_records"][k]])
        want = np.array([[r.primal_residual, r.dual_residual] for r in o1["records"]])
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12)
        to = one.trajectories()
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b{b}"
            np.testing.assert_allclose(tb[al], to[al], rtol=1e-9, atol=1e-12)


def test_gpu_c2_bench_fleet_blocks_stop_like_their_own_coordinators():
    """The C2 leg's own fleet (`bench.py` c2_admm: 1024 blocks = the 4096-room fleet, seed
    20261015 + 1, the reference's IPOPT settings, the example coordinator's stopping rule): at
    4096 rooms the room class runs the MAIN code object (more than four agents per CU), which a
    single-block run (small-fleet build) never touches.  The first block, the blocks that stop
    first and last, and a middle one each end at the iteration, with the residual history and
    coupling means, of a single-block run of that block alone."""
    N, kw = 10, dict(admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
    opts = {"ipopt": {}}
    big = ADMMFleet(bm.c2_fleet_classes(n_blocks=1024, N=N, seed=20261015 + 1, solver_options=opts))
    rooms = big.classes[0]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    assert rooms.n == 4096 and rooms.n > 4 * cus, "the room class must run the main build at this size"
    out = big.run_coordinated(0.4, **kw)
    its = np.asarray(out["block_iterations"])
    assert len(set(its.tolist())) > 1, its
    tb = big.trajectories()
    seed_block = {big.block_index(f"mDot1_coupling_b{b}"): b for b in range(1024)}
    for k in sorted({big.block_index("mDot1_coupling_b0"), int(np.argmin(its)), int(np.argmax(its)),
                     big.block_index("mDot1_coupling_b511")}):
        b = seed_block[k]
        one = ADMMFleet(bm.c2_fleet_classes(n_blocks=1, N=N, seed=20261015 + 1, block_offset=b, solver_options=opts))
        o1 = one.run_coordinated(0.4, **kw)
        assert its[k] == o1["iterations"], (b, its[k], o1["iterations"])
        got = np.array([[r.primal_residual, r.dual_residual] for r in out["block_records"][k]])
        want = np.array([[r.primal_residual, r.dual_residual] for r in o1["records"]])
        np.testing.assert_allclose(got, want, rtol=1e-7, atol=1e-12)
        to = one.trajectories()
        for i in range(4):
            al = f"mDot{i + 1}_coupling_b{b}"
            np.testing.assert_allclose(tb[al], to[al], rtol=1e-7, atol=1e-10)


def test_gpu_admm_golden_through_native_kernels():
    """The reference's own ConsensusVariable / ExchangeVariable outputs
    (`tests/golden/admm_golden.json`, produced by executing `admm_datatypes.py` itself,
    `tests/golden/make_golden.py`) fed straight through the HIP kernels: two mean /
    multiplier rounds over the active participants, residual norms, diffs, shifts."""
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "admm_golden.json")))
    ops = NativeADMMOps()

    def dev(a, dt=torch.float64):
        return torch.as_tensor(np.asarray(a), dtype=dt).cuda().contiguous()

    n_cons = n_exch = 0
    for case in gold:
        T, rho = case["T"], case["rho"]
        if case["type"] == "consensus":
            srcs = [s_ for s_ in case["sources"] if s_ in set(case["active"])]
            gs = dev([0, len(srcs)], torch.int32)
            mean, dmean = dev(np.zeros((1, T))), dev(np.zeros((1, T)))   # mean_trajectory = [0]
            LAM = dev([case["multipliers0"][k] for k in srcs])
            for rnd in (1, 2):
                X = dev([case[f"locals{rnd - 1}"][k] for k in srcs])
                mom = dev(np.zeros(ops.moments_size(1, 1, T)))
                ops.moments(1, 0, 1, T, gs, len(srcs), X, LAM, mean, mom)
                tot = mom[0:8]
                ops.finalize(0, 1, 0, 1, T, mom, None, None, rho, None, None, None, mean, dmean, tot)
                ops.consensus_multipliers(1, T, gs, len(srcs), X, mean, rho, None, None, LAM)
                torch.cuda.synchronize()
                np.testing.assert_allclose(mean.cpu().numpy()[0], case[f"mean{rnd}"], rtol=1e-13, atol=1e-15)
                np.testing.assert_allclose(dmean.cpu().numpy()[0], case[f"delta_mean{rnd}"], rtol=1e-12,
                                           atol=1e-15)
                np.testing.assert_allclose(np.sqrt(tot[0].item()), np.linalg.norm(case[f"primal{rnd}"]),
                                           rtol=1e-9, atol=1e-14)
                np.testing.assert_allclose(np.sqrt(tot[1].item()), np.linalg.norm(case[f"dual{rnd}"]),
                                           rtol=1e-9, atol=1e-12)
            lam = LAM.cpu().numpy()
            for i, k in enumerate(srcs):
                np.testing.assert_allclose(lam[i], case["multipliers2"][k], rtol=1e-12, atol=1e-12)
            ops.shift(T, 1, mean)
            ops.shift(T, 1, LAM)
            torch.cuda.synchronize()
            np.testing.assert_allclose(mean.cpu().numpy()[0], case["shifted_mean"], rtol=1e-13, atol=1e-15)
            lam = LAM.cpu().numpy()
            for i, k in enumerate(srcs):
                np.testing.assert_allclose(lam[i], case["shifted_multipliers"][k], rtol=1e-12, atol=1e-12)
            n_cons += 1
        else:
            srcs = case["sources"]
            gs = dev([0, len(srcs)], torch.int32)
            X = dev([case["locals0"][k] for k in srcs])
            mean, dmean = dev(np.zeros((1, T))), dev(np.zeros((1, T)))
            GM, DIFF, EX = dev([case["multiplier0"]]), dev(np.zeros((len(srcs), T))), dev([1], torch.int32)
            mom = dev(np.zeros(ops.moments_size(1, 1, T)))
            ops.moments(1, 0, 1, T, gs, len(srcs), X, None, mean, mom)
            tot = mom[0:8]
            ops.finalize(0, 1, 0, 1, T, mom, EX, GM, rho, None, None, None, mean, dmean, tot)
            ops.exchange_update(1, T, gs, len(srcs), X, mean, DIFF, GM, True, rho, None, None)
            torch.cuda.synchronize()
            np.testing.assert_allclose(mean.cpu().numpy()[0], case["mean1"], rtol=1e-13, atol=1e-15)
            np.testing.assert_allclose(dmean.cpu().numpy()[0], case["delta_mean1"], rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(GM.cpu().numpy()[0], case["multiplier1"], rtol=1e-13, atol=1e-12)
            diff = DIFF.cpu().numpy()
            for i, k in enumerate(srcs):
                np.testing.assert_allclose(diff[i], case["diffs1"][k], rtol=1e-12, atol=1e-15)
            np.testing.assert_allclose(np.sqrt(tot[0].item()), np.linalg.norm(case["primal1"]), rtol=1e-12)
            np.testing.assert_allclose(np.sqrt(tot[1].item()), np.linalg.norm(case["dual1"]), rtol=1e-9)
            ops.shift(T, 1, GM)
            ops.shift(T, 1, DIFF)
            torch.cuda.synchronize()
            np.testing.assert_allclose(GM.cpu().numpy()[0], case["shifted_multiplier"], rtol=1e-13, atol=1e-12)
            diff = DIFF.cpu().numpy()
            for i, k in enumerate(srcs):
                np.testing.assert_allclose(diff[i], case["shifted_diffs"][k], rtol=1e-12, atol=1e-15)
            n_exch += 1
    assert n_cons > 0 and n_exch > 0


def test_gpu_c4_fleet_at_scale_matches_local_round_with_c_oracle():
    """examples/exchange_admm scaled to 1024 agents on ONE exchange alias (1020 rooms with
    d~U(10,150), T0~U(296,303) + 4 supply units; rho=1e4, N=10, 3 LocalADMM iterations): the
    GPU fleet against `oracle/admm.local_round` (LocalADMM.process restated, one multiplier per
    agent) with the local solves done by the C IPM restatement over the host-compiled
    generated models (tests/admm_cases.CFleetOracle): exchange mean, every agent's local
    trajectory and multiplier."""
    N, iters = 10, 3
    classes = bm.c4_fleet_classes(n_rooms=1020, n_supply=4, N=N, seed=11)
    fl = ADMMFleet(classes)
    out = fl.run_local(penalty_factor=1e4, max_iterations=iters)
    assert out["converged_solves"] == 1024 * iters
    orc = CFleetOracle(classes, bm.TIGHT["ipopt"])
    state, hist = oadmm.local_round(orc.participation, orc.initial, orc, 1e4, 1, iters, T=N)
    np.testing.assert_allclose(fl.trajectories()["mDot_coupling"], hist[-1]["mDot_coupling"], rtol=RTOL, atol=1e-9)
    for cname, n in (("room", 1020), ("supply", 4)):
        loc, mult = fl.locals_of(cname, "mDot_out"), fl.multipliers_of(cname, "mDot_out")
        want_l = np.array([state["local"][(f"{cname}#{i}", "mDot_coupling")] for i in range(n)])
        want_m = np.array([state["mult"][(f"{cname}#{i}", "mDot_coupling")] for i in range(n)])
        np.testing.assert_allclose(loc, want_l, rtol=RTOL, atol=1e-7)   # at-bound entries: barrier distances
        np.testing.assert_allclose(mult, want_m, rtol=RTOL, atol=1e-5 * np.abs(want_m).max())


def test_gpu_c4_full_size_fleet_properties():
    """BASELINE.json configs[3] at its full size: examples/exchange_admm scaled to 16384 agents
    (13108 rooms + 3276 supply units, one exchange alias; rho=1e4, N=10, 15 LocalADMM
    iterations, the reference IPOPT settings), the bench's fleet.  Size-independent checks:
    every one of the 16384 x 15 local solves succeeds; the exchange mean is the mean of the
    agents' final local trajectories (the moment identity the segmented-sum kernels compute);
    the last multiplier update is lambda_15 - lambda_14 = rho * mean_15 (`admm.py:639-655`),
    lambda_14 taken from a 14-iteration run of the same fleet."""
    N, rho = 10, 1e4
    make = lambda: bm.c4_fleet_classes(n_rooms=13108, n_supply=3276, N=N, seed=20261015 + 4,  # noqa: E731
                                       solver_options=bm.REFERENCE)
    fl = ADMMFleet(make())
    out = fl.run_local(rho, max_iterations=15)
    assert out["converged_solves"] == 16384 * 15
    locs = np.vstack([fl.locals_of("room", "mDot_out"), fl.locals_of("supply", "mDot_out")])
    assert locs.shape == (16384, N)
    mean15 = fl.trajectories()["mDot_coupling"]
    # the kernel's segmented sums add 16384 signed terms in atomic (unordered) order
    np.testing.assert_allclose(mean15, locs.mean(axis=0), rtol=1e-12, atol=1e-12 * np.abs(locs).max())
    lam15 = fl.multipliers_of("room", "mDot_out")
    assert np.all(lam15 == lam15[0])   # one multiplier per alias: every participant's copy equal
    fl14 = ADMMFleet(make())
    fl14.run_local(rho, max_iterations=14)
    lam14 = fl14.multipliers_of("room", "mDot_out")
    np.testing.assert_allclose(lam15[0] - lam14[0], rho * mean15, rtol=1e-9, atol=1e-9 * rho * np.abs(mean15).max())


def test_gpu_c5_full_size_fleet_blocks_equal_their_own_runs():
    """BASELINE.json configs[4] at its full size: 342 three-zone blocks (1026 NARX zones +
    342 AHU + 342 CCA agents, one batched launch per class and ADMM iteration), 3 coordinated
    iterations: the first, a middle and the last block each equal a single-block fleet of that
    block alone (residual history and coupling means)."""
    N, kw = 24, dict(admm_iter_max=3, use_relative_tolerances=False, primal_tol=0.0, dual_tol=0.0)
    opts = bm.REFERENCE
    big = ADMMFleet(bm.c5_fleet_classes(n_blocks=342, N=N, seed=20261015 + 5, solver_options=opts))
    assert big.n_blocks == 342 and sum(c.n for c in big.classes) == 5 * 342
    out = big.run_coordinated(1.0, **kw)
    tb = big.trajectories()
    for b in (0, 171, 341):
        one = ADMMFleet(bm.c5_fleet_classes(n_blocks=1, N=N, seed=20261015 + 5, block_offset=b,
                                            solver_options=opts))
        o1 = one.run_coordinated(1.0, **kw)
        k = big.block_index(f"T_airin1_b{b}")
        got = np.array([[r.primal_residual, r.dual_residual] for r in out["block_records"][k]])
        want = np.array([[r.primal_residual, r.dual_residual] for r in o1["records"]])
        np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-12)
        to = one.trajectories()
        for pre in ("T_coupling", "T_coupling_ahu", "T_rucklauf", "T_airin"):
            for i in range(3):
                al = f"{pre}{i + 1}_b{b}"
                np.testing.assert_allclose(tb[al], to[al], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("crit", [(0, 1e-3, 1e-3, 2e-3, 0.05, -1.0, 2.0), (1, 0.05, 0.02, 1e-3, 1e-3, 1.5, 1.3)])
def test_gpu_block_stop_matches_restatement(crit):
    """``mpcx_admm_block_stop`` / ``mpcx_admm_block_expand`` against their numpy restatement
    (`oracle/cpu_fleet.py`, the host coordinator's rule) on random residual totals of 700
    blocks over 6 iterations: same freeze decisions and iteration counts, penalties, records
    and active counts (absolute criterion; relative criterion with penalty variation)."""
    from oracle.cpu_fleet import CpuFleetOps

    rng = np.random.default_rng(3)
    nb, its = 700, 6
    ops_g, ops_c = NativeADMMOps(), CpuFleetOps()
    state = {}
    for name, dev in (("gpu", "cuda"), ("cpu", "cpu")):
        f = lambda *a, **k: torch.zeros(*a, **k, device=dev)  # noqa: E731
        state[name] = dict(rho=torch.full((nb, 1), 0.4, dtype=torch.float64, device=dev),
                           act=torch.ones(nb, dtype=torch.int32, device=dev),
                           it=torch.full((nb,), its, dtype=torch.int32, device=dev),
                           rec=f(its * nb * 4, dtype=torch.float64), nact=f(its + 1, dtype=torch.int32),
                           clk=f(its + 1, dtype=torch.int64))
    idx = rng.integers(0, nb, 1500).astype(np.int32)
    part = (rng.random(1500) < 0.9).astype(np.int32)
    for it in range(1, its + 1):
        tot = np.abs(rng.normal(size=(nb, 8))) * np.array([1e-5, 1e-2, 1, 1, 1, 30, 30, 1]) * rng.random((nb, 1))
        for name, ops in (("gpu", ops_g), ("cpu", ops_c)):
            s = state[name]
            dev = "cuda" if name == "gpu" else "cpu"
            ops.block_stop(it, torch.as_tensor(tot.ravel(), device=dev), crit, s["rho"], s["act"], s["it"], s["rec"],
                           s["nact"], s["clk"])
            out_a = torch.zeros(1500, dtype=torch.int32, device=dev)
            out_r = torch.zeros(1500, dtype=torch.float64, device=dev)
            ops.block_expand(torch.as_tensor(idx, device=dev), s["act"], s["rho"], torch.as_tensor(part, device=dev),
                             out_a, out_r)
            s["exp"] = (out_a.cpu().numpy(), out_r.cpu().numpy())
        g, c = state["gpu"], state["cpu"]
        for k in ("act", "it", "nact"):
            np.testing.assert_array_equal(g[k].cpu().numpy(), c[k].cpu().numpy(), err_msg=k)
        np.testing.assert_allclose(g["rho"].cpu().numpy(), c["rho"].numpy(), rtol=1e-15)
        np.testing.assert_allclose(g["rec"].cpu().numpy(), c["rec"].numpy(), rtol=1e-14)
        np.testing.assert_array_equal(g["exp"][0], c["exp"][0])
        np.testing.assert_allclose(g["exp"][1], c["exp"][1], rtol=1e-15)
    assert 0 < int(state["cpu"]["nact"][1]) < nb          # some blocks stopped, some did not
    assert (state["gpu"]["clk"].cpu().numpy()[1:] >= state["gpu"]["clk"].cpu().numpy()[:-1]).all()


def test_gpu_stats_count_matches_restatement():
    """``mpcx_stats_count`` (C ABI v9, one launch per class and ADMM iteration instead of a chain of
    tensor ops) against its numpy restatement (`oracle/cpu_fleet.py`) on random stats records of
    5000 agents (statuses -4..3, restoration counts 0..3), with and without an active mask,
    accumulated over two calls."""
    from agentlib_mpc_amd.runtime.native import STATS_BYTES
    from oracle.cpu_fleet import CpuFleetOps

    rng = np.random.default_rng(11)
    n = 5000
    words = np.zeros((n, STATS_BYTES // 4), np.int32)
    words[:, 13] = rng.integers(-4, 4, n)  # status
    words[:, 15] = rng.integers(0, 4, n)   # n_restorations
    raw = words.view(np.uint8).ravel()
    act = (rng.random(n) < 0.7).astype(np.int32)
    got, want = {}, {}
    for name, ops, dev in (("gpu", NativeADMMOps(), "cuda"), ("cpu", CpuFleetOps(), "cpu")):
        st = torch.as_tensor(raw, device=dev)
        counts = torch.zeros(2, dtype=torch.int64, device=dev)
        ops.stats_count(n, st, None, counts)
        ops.stats_count(n, st, torch.as_tensor(act, device=dev), counts)
        (got if name == "gpu" else want)["c"] = counts.cpu().numpy()
    ok = (words[:, 13] == 0) | (words[:, 13] == 1)
    expect = [ok.sum() + (ok & (act != 0)).sum(), words[:, 15].sum() + words[:, 15][act != 0].sum()]
    np.testing.assert_array_equal(want["c"], expect)
    np.testing.assert_array_equal(got["c"], expect)


@pytest.mark.parametrize("n", [0, 1, 700, 5000, 16384])
def test_gpu_active_map_matches_restatement(n):
    """``mpcx_active_map`` (C ABI v11) against its numpy restatement (`oracle/cpu_fleet.py`): the
    active indices in increasing order, then -1, and the count."""
    from oracle.cpu_fleet import CpuFleetOps

    rng = np.random.default_rng(n)
    act = (rng.random(n) < 0.3).astype(np.int32)
    out = {}
    for name, ops, dev in (("gpu", NativeADMMOps(), "cuda"), ("cpu", CpuFleetOps(), "cpu")):
        amap = torch.full((n,), 7, dtype=torch.int32, device=dev)
        cnt = torch.zeros(1, dtype=torch.int32, device=dev)
        ops.active_map(n, torch.as_tensor(act, device=dev), amap, cnt)
        out[name] = (amap.cpu().numpy(), int(cnt.item()))
    np.testing.assert_array_equal(out["gpu"][0], out["cpu"][0])
    assert out["gpu"][1] == out["cpu"][1] == int(act.sum())
    np.testing.assert_array_equal(out["gpu"][0][:int(act.sum())], np.flatnonzero(act))


def test_gpu_mapped_launch_matches_full_launch(monkeypatch):
    """Coordinated rounds launch only the agents still active (``mpcx_active_map`` +
    ``mpcx_batch_solve_mapped``, C ABI v11; the code object chosen by the launch size, so the
    stragglers of a mostly converged fleet run the small-fleet build): a 256-block C2 fleet at
    the reference's settings over two closed-loop steps gives every block the stopping iteration,
    residual history and means of the same fleet launched whole (one launch of every agent, the
    converged ones skipped in the kernel).  The builds differ in FMA contraction (1e-12)."""
    N, kw = 10, dict(admm_iter_max=40, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
    runs = {}
    for mapped in (True, False):
        monkeypatch.setenv("MPCX_FLEET_MAP", "1" if mapped else "0")
        fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=256, N=N, seed=20261015 + 1, solver_options={"ipopt": {}}))
        assert fl.map_launch == mapped
        outs = []
        for step in range(2):
            if step:
                bm.advance_plant(fl, 60.0)
            outs.append(fl.run_coordinated(0.4, **kw))
        bounds = [c.bound for c in fl.classes]
        runs[mapped] = (outs, fl.trajectories(), bounds)
    (om, tm, bm_), (of, tf, _) = runs[True], runs[False]
    assert any(b < c.n for b, c in zip(bm_, fl.classes)), bm_   # the mapped fleet did shrink its launches
    for a, b in zip(om, of):
        np.testing.assert_array_equal(a["block_iterations"], b["block_iterations"])
        assert a["converged_solves"] == b["converged_solves"]
        for k in range(0, 256, 17):
            ga = np.array([[r.primal_residual, r.dual_residual] for r in a["block_records"][k]])
            gb = np.array([[r.primal_residual, r.dual_residual] for r in b["block_records"][k]])
            np.testing.assert_allclose(ga, gb, rtol=1e-8, atol=1e-12)
    for al in tm:
        np.testing.assert_allclose(tm[al], tf[al], rtol=1e-8, atol=1e-11)


def test_gpu_fused_moves_match_one_launch_per_move(monkeypatch):
    """A class's per-iteration row moves -- every slot's mean / multiplier columns and the block
    penalty into p, every slot's local trajectory out of w -- as one scatter and one gather launch
    (``mpcx_scatter_rows_multi`` / ``mpcx_gather_rows_multi``, C ABI v12) are the same copies as one
    launch per move: a 64-block C2 fleet (a room class with one slot, an air-handler class with
    four) over two closed-loop steps, and the C4 exchange fleet's LocalADMM round, come out bit for
    bit equal."""
    N, kw = 10, dict(admm_iter_max=20, use_relative_tolerances=False, primal_tol=0.002, dual_tol=0.1)
    runs = {}
    for fused in (True, False):
        monkeypatch.setenv("MPCX_FLEET_FUSED", "1" if fused else "0")
        fl = ADMMFleet(bm.c2_fleet_classes(n_blocks=64, N=N, seed=20261015 + 7, solver_options={"ipopt": {}}))
        assert fl.fused_moves == fused
        outs = []
        for step in range(2):
            if step:
                bm.advance_plant(fl, 60.0)
            outs.append(fl.run_coordinated(0.4, **kw))
        ex = ADMMFleet(bm.c4_fleet_classes(n_rooms=48, n_supply=12, N=10, seed=20261015 + 4,
                                           solver_options={"ipopt": {}}))
        ex.run_local(1e4, max_iterations=3, record_residuals=True)
        runs[fused] = (outs, fl.trajectories(), fl.X.cpu().numpy(), ex.X.cpu().numpy(), ex.trajectories())
    (of, tf, xf, ef, etf), (ou, tu, xu, eu, etu) = runs[True], runs[False]
    for a, b in zip(of, ou):
        np.testing.assert_array_equal(a["block_iterations"], b["block_iterations"])
    np.testing.assert_array_equal(xf[:-1], xu[:-1])   # the last row is the scratch row
    np.testing.assert_array_equal(ef[:-1], eu[:-1])
    for al in tf:
        np.testing.assert_array_equal(tf[al], tu[al])
    for al in etf:
        np.testing.assert_array_equal(etf[al], etu[al])


def test_gpu_collective_rccl_transport_one_rank(tmp_path):
    """C ABI v14 on the GPU: the ADMM iteration's all-reduce issued by the library on an
    RCCL communicator.  One rank (the box has one GPU; a communicator's ranks must sit on distinct
    GPUs): (1) the fleet driver's path -- a one-rank ``nccl`` process group, the library's own
    communicator made from PyTorch's loaded RCCL (``runtime/collective.py``), the sum over one rank
    leaves the buffer as it is and the library counts the call; (2) a C caller's path --
    ``mpcx_rccl_comm_init_file`` (shared-file bootstrap of the unique id), ``mpcx_allreduce_register``,
    ``mpcx_admm_allreduce`` on a HIP stream, ``mpcx_rccl_comm_destroy``."""
    import ctypes
    import torch.distributed as dist

    from agentlib_mpc_amd.runtime import collective, native

    lib = native.load_library()
    dist.init_process_group("nccl", init_method=f"file://{tmp_path / 'pg'}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        coll = collective.Collective(dist, None, torch.device("cuda"))
        assert coll.kind == "rccl" and collective.kind() == native.COLLECTIVE_RCCL
        buf = torch.arange(1.0, 41.0, dtype=torch.float64, device="cuda")
        coll.bind(buf)
        c0 = collective.calls()
        for _ in range(5):
            coll.allreduce(33)
        torch.cuda.synchronize()
        assert collective.calls() - c0 == 5
        np.testing.assert_array_equal(buf.cpu().numpy(), np.arange(1.0, 41.0))
    finally:
        lib.mpcx_allreduce_unregister()
        dist.destroy_process_group()
    path = collective.loaded_rccl_path()
    cpath = path.encode() if path else None
    comm = ctypes.c_void_p()
    assert lib.mpcx_rccl_comm_init_file(cpath, str(tmp_path / "rccl_id").encode(), 1, 0, 10000, ctypes.byref(comm)) == 0
    try:
        assert lib.mpcx_allreduce_register(comm, cpath) == 0
        x = torch.full((17,), 2.5, dtype=torch.float64, device="cuda")
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            assert lib.mpcx_admm_allreduce(ctypes.c_void_p(x.data_ptr()), 17, ctypes.c_void_p(s.cuda_stream)) == 0
        s.synchronize()
        np.testing.assert_array_equal(x.cpu().numpy(), np.full(17, 2.5))
    finally:
        assert lib.mpcx_rccl_comm_destroy(cpath, comm) == 0
    assert lib.mpcx_allreduce_kind() == native.COLLECTIVE_NONE

def test_gpu_dedicated_streams_overlap():
    """C ABI v15: two streams from mpcx_stream_create_dedicated (hardware queues of their own) run
    a spin kernel each at the same time -- ordinary streams of a process share the runtime's few
    hardware queues, on which the C2 rooms' and air handlers' solves ran one after the other (r06,
    scripts/queue_probe.py)."""
    import time

    from agentlib_mpc_amd.runtime.native import dedicated_streams

    a, b = dedicated_streams(2, "cuda")
    assert a.cuda_stream != b.cuda_stream
    cycles = 4_000_000

    def run(streams):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for s in streams:
            with torch.cuda.stream(s):
                torch.cuda._sleep(cycles)
        torch.cuda.synchronize()
        return time.perf_counter() - t

    run([a, b])  # warm-up (queue creation)
    one = min(run([a]) for _ in range(3))
    two = min(run([a, b]) for _ in range(3))
    print(f"one spin {one * 1e3:.3f} ms, two on dedicated streams {two * 1e3:.3f} ms")
    assert two < 1.5 * one, (one, two)
    assert dedicated_streams(2, "cuda")[0] is a  # the process-wide pool



def test_gpu_fused_bookkeeping_matches_per_class_launches():
    """C ABI v15: mpcx_admm_block_expand_multi / mpcx_stats_count_multi (one launch for the groups
    and every class) give exactly what one mpcx_admm_block_expand / mpcx_stats_count per class does
    -- random block maps, participation masks, freeze masks and solver stats."""
    from agentlib_mpc_amd.runtime.native import STATS_BYTES

    ops = NativeADMMOps()
    rng = np.random.default_rng(7)
    dev = torch.device("cuda")
    nb = 37
    active_b = torch.as_tensor(rng.integers(0, 2, nb).astype(np.int32), device=dev)
    rho_b = torch.as_tensor(rng.uniform(0.1, 10.0, (nb, 1)), device=dev)
    sizes = [1000, 257, 64, 1]
    entries, ref = [], []
    for k, n in enumerate(sizes):
        idx = torch.as_tensor(rng.integers(0, nb, n).astype(np.int32), device=dev)
        part = None if k % 2 else torch.as_tensor(rng.integers(0, 2, n).astype(np.int32), device=dev)
        oa, orho = torch.full((n,), -7, dtype=torch.int32, device=dev), None
        if k == 0:
            orho = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        entries.append((idx, part, oa, orho))
        ra = torch.full((n,), -7, dtype=torch.int32, device=dev)
        rr = None if orho is None else torch.full((n,), -1.0, dtype=torch.float64, device=dev)
        ops.block_expand(idx, active_b, rho_b if rr is not None else None, part, ra, rr)
        ref.append((ra, rr))
    ops.run_plan(ops.expand_plan(entries, active_b, rho_b))
    torch.cuda.synchronize()
    for (idx, part, oa, orho), (ra, rr) in zip(entries, ref):
        assert torch.equal(oa, ra)
        if orho is not None:
            assert torch.equal(orho, rr)
    stats, counts_ref = [], torch.zeros(2, dtype=torch.int64, device=dev)
    for n in sizes:
        raw = np.zeros((n, STATS_BYTES // 4), np.int32)
        st = torch.as_tensor(raw.reshape(-1).view(np.uint8), device=dev)
        words = st.view(torch.int32).view(n, STATS_BYTES // 4)
        act = torch.as_tensor(rng.integers(0, 2, n).astype(np.int32), device=dev)
        stats.append((n, st, act, words))
    # statuses and restoration counts through the native stats layout (mpcx_stats: status and
    # n_restorations fields), written via the record's dtype
    from agentlib_mpc_amd.runtime.native import stats_array
    for n, st, act, _ in stats:
        arr = stats_array(st.cpu().numpy().tobytes()).copy()
        arr["status"] = rng.integers(-3, 3, n)
        arr["n_restorations"] = rng.integers(0, 4, n)
        st.copy_(torch.as_tensor(np.frombuffer(arr.tobytes(), np.uint8).copy(), device=dev))
        ops.stats_count(n, st, act, counts_ref)
    counts = torch.zeros(2, dtype=torch.int64, device=dev)
    ops.run_plan(ops.stats_plan([(n, st, act) for n, st, act, _ in stats], counts))
    torch.cuda.synchronize()
    assert torch.equal(counts, counts_ref), (counts, counts_ref)
    assert int(counts_ref[0]) > 0 and int(counts_ref[1]) > 0
