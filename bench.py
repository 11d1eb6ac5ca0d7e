"""Benchmark: converged MPC solves/s on a synthetic fleet (BASELINE.json C3).

Workload: one_room model of `examples/one_room_mpc/physical/simple_mpc.py`
(backend "casadi", direct collocation, Legendre d=2, N=15, ts=300 s); per agent
T0~U(291.15,301.15), load~U(50,250), T_in~U(289.15,291.15),
T_upper~U(294.15,296.15), u_prev~U(0,0.05) from numpy default_rng(20261015+2+rank);
cold start.  One step = one batched solve of every agent on the GPU (the
initial guess is re-copied inside the timed region).  Solver settings: the
reference's IPOPT defaults (``--solver reference``, `casadi_utils.py:197-206`:
tol 1e-4, max_iter 100, acceptable_tol 0.1 over acceptable_iter 5,
acceptable_constr_viol_tol 1, acceptable_compl_inf_tol 1); a solve counts as
converged when it ends Solve_Succeeded or Solved_To_Acceptable_Level, IPOPT's two
success states.  ``--solver tight`` (tol ``--tol``, no acceptable stop) is the
parity setting.

Multi-GPU (torch.distributed, one process per GPU): every rank solves its own
fleet slice (``--agents`` per GPU, weak scaling, no data-path collective);
barrier + synchronize bracket the timed steps and the max time over ranks is
reported.

Extra JSON fields: ``roofline`` for the dominant kernel (mpcx_ipm_solve; kernel time measured
with HIP events on the launch stream; ``roofline_block``: bound "hbm" -- the counters show the
memory side as the limit -- with the algorithmic bytes as ``achieved``, the counted bytes as
``traffic`` / ``memory_side`` and the algorithmic FP64 flops beside them) and ``cpu_baseline``
(oracle timed on host cores on a bounded sample, rank 0, N=1 only).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings

# the reference models' objective-formulation deprecation notice (models/casadi_model.py, as the
# reference warns) fires once per model build -- dozens per run, which pushed the bench line out of
# the driver's captured output tail (BENCH_r05.json)
warnings.filterwarnings("ignore", message="Model uses the deprecated objective formulation")

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "agentlib-mpc_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = "converged MPC solves/sec (whole node) at N agents; ADMM iters/sec to consensus"
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 vector peak (spec)
PEAK_HBM_GBS = 8000.0
MEASURED_HBM_GBS = 6300.0  # MI355X_MICROARCH.md: ~6.3 TB/s achievable


def fleet_values(n, seed):
    rng = np.random.default_rng(seed)
    return {
        "T": rng.uniform(291.15, 301.15, n),
        "load": rng.uniform(50.0, 250.0, n),
        "T_in": rng.uniform(289.15, 291.15, n),
        "T_upper": rng.uniform(294.15, 296.15, n),
        "mDot": rng.uniform(0.0, 0.05, n),
    }


def flops_model(gen, stats):
    """Algorithmic FP64 flops of one batched solve (sum over agents)."""
    d = gen.dims
    N, NX, NV, NG = d["N"], d["NX"], d["NV"], d["NG"]
    NB = NV + NX + NG
    NW = NX + N * (NV + NX)
    M = N * NG
    # factorisation: the generated sparse static elimination per stage (its op count),
    # dense Bunch-Kaufman on the stages it rejected (stats n_dense_stages: bordered
    # packed system, NI pivots), the nx-block chain
    nmu = len(gen.bordered_rows)
    ni, nloc = NV + NG - nmu, NV + NG + NX + nmu
    f_dense_stage = sum((nloc + 1 - k) * (nloc + 2 - k) for k in range(ni)) + 2.0 * ni * (NX + nmu + NX + 1) * ni
    f_chain = N * (2.0 * (NX + nmu) ** 3 + 4.0 * (NX + nmu) ** 2 * NX)
    f_fact = N * (gen.elim.flops if gen.elim is not None else f_dense_stage) + f_chain
    f_solve = N * (2.0 * (NV + NG - len(gen.bordered_rows)) * (2 * NX + len(gen.bordered_rows))
                   + 4.0 * (NX + len(gen.bordered_rows)) ** 2)  # u = u0 - Z [x_k, c_k]; chain sweeps
    f_fg = N * gen.flops["fg"]
    f_gj = N * gen.flops["gj"]
    f_h = N * gen.flops["hess"]
    f_vec = 60.0 * (NW + M)
    it = stats["iter"].astype(float)
    dense = stats.get("dense", 0.0)
    tot = (stats["fact"] * f_fact + dense * f_dense_stage + (it + 1) * f_solve + (it + 2) * f_gj + it * f_h
           + (stats["trials"] + 1) * (f_fg + 10.0 * (NW + M)) + it * f_vec)
    return float(tot.sum())


def solver_settings(args):
    """(product solver_options, oracle IPOPT options) of the selected setting."""
    if args.solver == "reference":
        return {"ipopt": {}}, dict(tol=1e-4, max_iter=100, acceptable_tol=0.1, acceptable_iter=5,
                                   acceptable_constr_viol_tol=1.0, acceptable_compl_inf_tol=1.0)
    return ({"ipopt": {"tol": args.tol, "max_iter": 500, "acceptable_iter": 0}},
            dict(tol=args.tol, max_iter=500, acceptable_iter=0))


def cpu_baseline(p, lbw, ubw, w0, ipopt, min_seconds=10.0, max_repeats=200):
    """C restatement of the oracle IPM (oracle/c/ipm_oracle.c), OpenMP over the
    host cores allotted to this process (OMP_NUM_THREADS), on the rank-0 fleet,
    repeated until at least ``min_seconds`` of wall time (a bounded sample)."""
    from oracle import cbuild

    threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count() or 1)
    cbuild.build()
    ok = 0
    repeats = 0
    t0 = time.perf_counter()
    opts = dict(ipopt)
    tol, max_iter = opts.pop("tol"), opts.pop("max_iter")
    while repeats < max_repeats and (repeats == 0 or time.perf_counter() - t0 < min_seconds):
        _, _, n_ok = cbuild.solve_room_fleet(p, lbw, ubw, w0, tol=tol, max_iter=max_iter, threads=threads,
                                             **opts)
        ok += n_ok
        repeats += 1
    dt = time.perf_counter() - t0
    return {"value": ok / dt, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{repeats} x the rank-0 C3 fleet ({p.shape[0]} agents, same inputs and IPOPT settings "
                      f"{ipopt}) "
                      f"with oracle/c/ipm_oracle.c (IPOPT restatement, block-tridiagonal LDL^T, "
                      f"gcc -O3 -march=native, OpenMP {threads} threads): {dt:.2f} s wall"}


def pmc_fp64(code_object: str, n_agents: int, kernel_ms: float):
    """FP64 utilisation of the bench kernel from the committed rocprofv3 instruction-counter
    passes (``profiles/*/*/pmc_fp64_c3.json``, scripts/gpu_pmc.sh): FP64 VALU lane-ops issued
    (64 x (ADD + MUL + 2 FMA + TRANS) wave instructions, an upper bound: masked lanes still
    take the issue slot) and FP64 MFMA flops per launch, over this run's kernel time, against
    the FP64 peak; plus the wave-cycle split (VALU issue / any issue / waiting).  Same code
    object and fleet size only; otherwise None."""
    import glob

    if n_agents != 4096:
        return None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "*", "pmc_fp64_c3.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("code_object") == code_object:
            issued = (d["fp64_valu_flops_per_launch_upper"] + d["fp64_mfma_flops_per_launch"]) / (kernel_ms * 1e-3) / 1e12
            return {"issued_tflops_upper": issued, "issued_frac_upper": issued / PEAK_FP64_TFLOPS,
                    "fp64_share_of_valu_insts": d["fp64_share_of_valu_insts"],
                    "wave_cycle_split": d.get("wave_cycle_split"), "source": os.path.relpath(path, ROOT)}
    return None


def roofline_block(kernel_ms, io_bytes, flops, traffic, traffic_src, fp64_pmc):
    """``roofline`` of the C3 launch (the label follows the counters).

    bound "hbm": the rocprofv3 counters put the kernel on the memory side -- FETCH_SIZE + WRITE_SIZE
    bytes per launch at ~60 % of the 8 TB/s spec (FETCH_SIZE doubled: calibrated on known byte counts
    at 4, 8 and 16 B per lane, profiles/r06/s1/fetch_calib.json), waves parked on memory half their
    cycles, VALU issue ~17 % (profiles/r05/final2/pmc_fp64_c3.json).  ``achieved`` / ``frac``: the
    ALGORITHMIC bytes of a launch (its inputs and outputs) over the kernel time -- tiny,
    because the traffic is the solver's per-agent workspace (97 KB, re-streamed every IPM iteration,
    DESIGN §3) and not the problem's data; ``memory_side``: the counted bytes over the same time;
    ``fp64``: the algorithmic flops (generated-code op counts x per-agent counters) over that time."""
    ks = kernel_ms * 1e-3
    achieved = io_bytes / ks / 1e9
    mem = None
    if traffic:
        gbs = traffic / ks / 1e9
        mem = {"bytes_per_launch": traffic, "achieved": gbs, "unit": "GB/s", "frac_of_peak": gbs / PEAK_HBM_GBS,
               "frac_of_measured_max": gbs / MEASURED_HBM_GBS, "traffic_over_algorithmic": traffic / io_bytes,
               "fetch_size_factor": 2.0, "calibration": "profiles/r06/s1/fetch_calib.json", "source": traffic_src}
    fp = flops / ks / 1e12
    return {
        "bound": "hbm",
        "achieved": achieved,
        "peak": PEAK_HBM_GBS,
        "unit": "GB/s",
        "frac": achieved / PEAK_HBM_GBS,
        "traffic": traffic,
        "traffic_source": traffic_src,
        "memory_side": mem,
        "fp64": {"achieved": fp, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": fp / PEAK_FP64_TFLOPS,
                 "flops_per_launch": flops, "pmc": fp64_pmc},
        "algorithmic_io_bytes": io_bytes,
        "kernel": "mpcx_ipm_solve",
        "kernel_ms": kernel_ms,
        "note": "algorithmic bytes = the launch's NLP inputs and outputs (p, bounds, guess, solution, multipliers, "
                "stats); the counted traffic is the per-agent workspace every IPM iteration streams (its vectors, "
                "stage derivatives, compact stage images, back-substitution operators), which 16 agents per CU "
                "cannot keep in LDS (DESIGN §3, §5); FP64 work: generated-code op counts of the stage "
                "evaluations, the sparse static stage elimination, dense fallback stages and the state chain",
    }


def pmc_traffic(code_object: str, n_agents: int):
    """HBM bytes per launch of the bench kernel from the committed rocprofv3 PMC
    passes (``profiles/*/*/pmc_traffic_c3.json``: FETCH_SIZE and WRITE_SIZE in
    separate runs, FETCH_SIZE doubled as the MI355X guide prescribes for gfx950).
    Only a summary taken on the same code object and fleet size is used;
    otherwise None (PMC counters cannot be read inside the timed process)."""
    import glob

    if n_agents != 4096:
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "*", "pmc_traffic_c3.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        if d.get("code_object") == code_object:
            return float(d["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def admm_bench(args, world, rank, dev):
    """C4 (BASELINE.json configs[3]): decentralised exchange ADMM (LocalADMM semantics,
    examples/exchange_admm: MS-Euler, N=10, ts=120, rho=1e4, 15 iterations) on a fleet of
    ``--admm-agents`` agents IN TOTAL (rooms:supply = 4:1) split over the GPUs (strong
    scaling: the config is a fixed 16384-agent fleet), all on ONE exchange alias spanning
    the ranks: one RCCL all-reduce per ADMM iteration."""
    import torch
    import torch.distributed as dist
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    n = args.admm_agents
    n_sup = n // 5
    opts, _ = solver_settings(args)
    classes = bm.c4_fleet_classes(n_rooms=n - n_sup, n_supply=n_sup, N=10, seed=20261015 + 4,
                                  solver_options=opts, rank=rank, world=world)
    n_local = sum(c.n for c in classes)
    fleet = ADMMFleet(classes, device=dev, comm="default" if world > 1 else None)
    for c in classes:
        c.native.reserve(c.n)
    fleet.run_local(1e4, max_iterations=1, record_residuals=False)  # warm-up (code objects, RCCL)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    out = fleet.run_local(1e4, max_iterations=args.admm_iters, record_residuals=False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    t = torch.tensor([wall, float(out["converged_solves"])], dtype=torch.float64, device=dev)
    if world > 1:
        w = t[:1].clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0] = w[0]
    wall, ok = float(t[0]), float(t[1])
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        ns = n  # the whole fleet (15 iterations of 16384 C IPM solves: a few seconds on 16 cores)
        sample = bm.c4_fleet_classes(n_rooms=ns - ns // 5, n_supply=ns // 5, N=10, seed=20261015 + 4,
                                     solver_options=opts)
        cpu = admm_cpu_baseline(sample, lambda fl: fl.run_local(1e4, max_iterations=args.admm_iters,
                                                                record_residuals=False), n, "C4 LocalADMM")
    return {
        "cpu_baseline": cpu,
        "workload": "C4: exchange ADMM (LocalADMM), examples/exchange_admm rooms+supply 4:1, MS-Euler "
                    "N=10 ts=120 rho=1e4, one exchange alias spanning all GPUs",
        "scaling": "strong", "agents_total": n, "agents_rank0": n_local, "admm_iterations": args.admm_iters,
        "admm_iters_per_s": args.admm_iters / wall,
        "agent_solves_per_s": ok / wall,
        "converged_fraction": ok / (n * args.admm_iters),
        "ms_per_admm_iteration": wall / args.admm_iters * 1e3,
        "allreduce_per_iteration": 1 if world > 1 else 0,
        "allreduce_doubles": fleet.reduce_len if world > 1 else 0,
        **_restorations(out["restorations"], world, dev),
    }


def nn_bench(args, world, rank, dev):
    """C5 (BASELINE.json configs[4]): ``--nn-zones`` three-zone NARX room agents per GPU
    (two ANNs BN->Dense(32,sigmoid)->Dense(1), backend casadi_admm_nn, N=24, ts=1800),
    one batched local ADMM solve of the whole fleet per step (first iteration:
    z-bar = initial coupling values, lambda = 0), cold start."""
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs

    n = args.nn_zones
    be, cv = bm.room_nn(solver_options=solver_settings(args)[0])
    prob = be.problem
    rng = np.random.default_rng(20261015 + 5 + rank)
    vals = {"T_air": rng.uniform(292.0, 297.0, n), "d": rng.uniform(50.0, 200.0, n),
            "T_amb": rng.uniform(295.0, 303.0, n), "Q_rad": rng.uniform(0.0, 50.0, n)}
    p, lbw, ubw, w0 = prob.to_kernel(*fleet_nlp_inputs(prob, cv, vals))
    stats, wall, kernel_ms = _timed_batch(be, prob, p, lbw, ubw, w0, n, args, dev)
    ok = sum(1 for s in stats if s["success"])
    return {
        "workload": "C5: three-zone NARX room agents (casadi_admm_nn, 2 ANNs 9/8->32 sigmoid->1, "
                    "N=24 ts=1800, lifted lag window), one batched local ADMM solve per step",
        "zones_per_gpu": n, "nlp": prob.nlp.nlp_dims(),
        "kernel_nlp": {"nw": prob.nlp.kernel_nw, "ng": prob.nlp.kernel_ng, "np": prob.nlp.kernel_np},
        "solves_per_s": ok * args.steps / wall, "converged_fraction": ok / n,
        "mean_ipm_iterations": float(np.mean([s["iter_count"] for s in stats])),
        "ipm_iterations_p50_p99_max": [float(np.percentile([s["iter_count"] for s in stats], q)) for q in (50, 99, 100)],
        "statuses": sorted({int(s["status"]) for s in stats}),
        "mean_factorizations": float(np.mean([s["n_factorizations"] for s in stats])),
        "restorations_last_step": int(sum(s["n_restorations"] for s in stats)),
        "soft_restorations_last_step": int(sum(s["n_soft_restorations"] for s in stats)),
        "block_chain_fraction": float(np.sum([s["n_block_chain"] for s in stats]) /
                                      max(1, np.sum([s["n_factorizations"] for s in stats]))),
        "kernel_ms": kernel_ms,
    }


def _timed_batch(be, prob, p, lbw, ubw, w0, n, args, dev):
    """W untimed + K timed batched solves of one fleet (cold start each step);
    returns (per-agent stats of the last step, wall seconds, kernel ms per step)."""
    import torch
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts

    native = be._native()
    native.reserve(n)
    T = lambda a: torch.as_tensor(a, device=dev).contiguous()  # noqa: E731
    tp, tl, tu, tw0 = T(p), T(lbw), T(ubw), T(w0)
    tw = torch.empty_like(tw0)
    lam = torch.empty((n, prob.nlp.kernel_ng), dtype=torch.float64, device=dev)
    st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        tw.copy_(tw0)
        native.solve(tp, tl, tu, tw, lam_g=lam, stats=st, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return stats_to_dicts(st.cpu().numpy().tobytes()), wall, ev0.elapsed_time(ev1) / args.steps


def c3_strong_bench(args, world, rank, dev):
    """C3 at a FIXED fleet (BASELINE.json configs[2]: the synthetic 4096-room fleet on 1/2/4/8
    GPUs): ``--agents`` agents in total (the same agents as the one-GPU fleet), each rank
    solving its contiguous share; no collective on the data path.  Reported beside the
    weak-scaling headline (which keeps ``--agents`` per GPU)."""
    import torch
    import torch.distributed as dist
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs

    be, cv = bm.one_room(solver_options=solver_settings(args)[0])
    prob = be.problem
    lo, hi = bm.split_range(args.agents, rank, world)
    vals = {k: v[lo:hi] for k, v in fleet_values(args.agents, 20261015 + 2).items()}
    p, lbw, ubw, w0 = fleet_nlp_inputs(prob, cv, vals)
    if world > 1:
        dist.barrier()
    stats, wall, kernel_ms = _timed_batch(be, prob, p, lbw, ubw, w0, hi - lo, args, dev)
    ok = sum(1 for s in stats if s["success"])
    t = torch.tensor([wall, float(ok)], dtype=torch.float64, device=dev)
    if world > 1:
        w = t[:1].clone()
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t[0] = w[0]
    return {"workload": "C3 fixed fleet split over the GPUs", "scaling": "strong", "agents_total": args.agents,
            "agents_rank0": hi - lo, "solves_per_s": float(t[1]) * args.steps / float(t[0]),
            "ms_per_step": float(t[0]) / args.steps * 1e3, "kernel_ms_rank0": kernel_ms}


def mhe_bench(args, world, rank, dev):
    """Moving horizon estimation fleet (backend casadi_mhe, `examples/Estimators/
    mhe_example.py`: RNGRoom, N=15, ts=200, Legendre d=2, estimating the capacity
    factor in [5, 6]): ``--mhe-agents`` estimators per GPU, each with its own
    noisy zone-temperature history (true factor 5.5, noise sigma 0.05 K), one
    batched solve per step, cold start."""
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs

    n = args.mhe_agents
    be, cv = bm.mhe_room(solver_options=solver_settings(args)[0])
    prob = be.problem
    p, lbw, ubw, w0 = fleet_nlp_inputs(prob, cv, {"weight_T": np.ones(n)})
    rng = np.random.default_rng(20261015 + 6 + rank)
    meas = prob.nlp.par_groups["measured_states"].index  # [2, N*d] positions in p
    p[:, meas[0]] += rng.normal(scale=0.05, size=(n, meas.shape[1]))
    p, lbw, ubw, w0 = prob.to_kernel(p, lbw, ubw, w0)
    stats, wall, kernel_ms = _timed_batch(be, prob, p, lbw, ubw, w0, n, args, dev)
    ok = sum(1 for s in stats if s["success"])
    return {
        "workload": "MHE: RNGRoom estimator fleet (casadi_mhe, collocation Legendre d=2, N=15, ts=200, "
                    "theta in [5,6], noisy T history), one batched solve per step",
        "agents_per_gpu": n, "nlp": prob.nlp.nlp_dims(),
        "kernel_nlp": {"nw": prob.nlp.kernel_nw, "ng": prob.nlp.kernel_ng, "np": prob.nlp.kernel_np},
        "solves_per_s": ok * args.steps / wall, "converged_fraction": ok / n,
        "mean_ipm_iterations": float(np.mean([s["iter_count"] for s in stats])),
        "ipm_iterations_p50_p99_max": [float(np.percentile([s["iter_count"] for s in stats], q)) for q in (50, 99, 100)],
        "restorations_last_step": int(sum(s["n_restorations"] for s in stats)),
        "soft_restorations_last_step": int(sum(s["n_soft_restorations"] for s in stats)),
        "factorisation": "stage-parallel, continuity rows bordered into the chain (DESIGN 2.1)"
                         if prob.gen.bordered_rows else "stage-parallel",
        "block_chain_fraction": float(np.sum([s["n_block_chain"] for s in stats]) /
                                      max(1, np.sum([s["n_factorizations"] for s in stats]))),
        "kernel_ms": kernel_ms,
    }


def c2_admm_bench(args, world, rank, dev):
    """C2 scaled (BASELINE.json configs[1]): ``--c2-blocks`` blocks per GPU of
    (4 rooms + air handler) of `examples/4_Room_ADMM_Coordinator`, coordinated
    consensus ADMM run to consensus with the example's coordinator settings
    (`configs/coordinator.json`: rho=0.4, admm_iter_max=40, absolute criterion
    primal_tol=0.002, dual_tol=0.1), reference IPOPT defaults for the local solves;
    the consensus groups are block-local, so ranks need no data-path collective
    beyond the residual totals.  Every block stops on its own residuals, as its own
    coordinator would (converged blocks are frozen while the rest iterate)."""
    import torch
    import torch.distributed as dist
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    nb = args.c2_blocks
    lo, hi = bm.split_range(nb, rank, world)
    make = lambda n, off=rank * 8: bm.c2_fleet_classes(n_blocks=n, N=10, seed=20261015 + 1,  # noqa: E731
                                                      block_offset=off, solver_options={"ipopt": {}})
    _warm_fleet(make, lambda fl: fl.run_coordinated(0.4, admm_iter_max=2, use_relative_tolerances=False,
                                                    primal_tol=0.002, dual_tol=0.1), world, dev)
    classes = make(hi - lo, lo)
    fleet = ADMMFleet(classes, device=dev, comm="default" if world > 1 else None)
    for c in classes:
        c.native.reserve(c.n)
    loop = _closed_loop(fleet, lambda: fleet.run_coordinated(0.4, admm_iter_max=40, use_relative_tolerances=False,
                                                              primal_tol=0.002, dual_tol=0.1),
                        args.admm_steps, 60.0, 5, world, dev)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the GPU leg's fleet and closed loop (a few x 40 ADMM iterations of 5120 C IPM solves:
        # ~30 s on 16 host cores)
        sample = bm.c2_fleet_classes(n_blocks=nb, N=10, seed=20261015 + 1, solver_options={"ipopt": {}})
        cpu = admm_cpu_baseline_closed_loop(
            sample, lambda fl: fl.run_coordinated(0.4, admm_iter_max=40, use_relative_tolerances=False,
                                                  primal_tol=0.002, dual_tol=0.1),
            5 * nb, "C2 coordinated, to each block's stopping rule", args.admm_steps, 60.0)
    return {
        "workload": "C2 scaled: 4-room + air-handler blocks (casadi_admm collocation d=3, N=10, ts=60), "
                    "coordinated consensus, rho=0.4, abs tol 0.002/0.1, iter max 40, per-block stopping; "
                    "the north-star 4096-room fleet (1024 blocks) split over the GPUs",
        "scaling": "strong", "blocks_total": nb, "rooms_total": 4 * nb, "agents_total": 5 * nb,
        "blocks_rank0": hi - lo if rank == 0 else None,
        "allreduce_doubles": fleet.reduce_len if world > 1 else 0,
        **loop,
        "cpu_baseline": cpu,
    }


def _closed_loop(fleet, run, steps, ts, agents_per_block, world, dev):
    """``steps`` control steps of a coordinated fleet, as the reference's coordinator runs
    them (`admm_coordinator.py:259-321`): each step shifts means and multipliers by one
    interval and iterates every block to its own stopping rule (or the iteration cap) from
    the agents' resident warm starts; between the steps the synthetic plant moves every
    zone to its predicted state at ``ts`` (``benchmarks.advance_plant``: new measurements,
    untimed).  Each step is timed on its own (barrier + synchronize on both sides).  The leg
    reports the per-step figures and, over the whole sequence, ADMM iterations/s = all steps'
    fleet-loop iterations / all steps' wall time (r05: the median over the steps sat between
    the slow cold steps and the fast warm ones and moved by 40 % between boxes) and block
    iterations/s = all blocks' own iterations / the same wall time (the fleet-loop rate rises
    as blocks freeze; the block rate counts the work each coordinator did).  ``dev`` "cpu": the
    same loop on the host fleet (the CPU baseline runs the identical step sequence)."""
    import torch
    import torch.distributed as dist
    from agentlib_mpc_amd import benchmarks as bm

    cuda = torch.device(dev).type == "cuda"
    per = []
    rest = 0
    for step in range(max(int(steps), 1)):
        if step:
            bm.advance_plant(fleet, ts)
        if cuda and os.environ.get("MPCX_BENCH_WAKE") == "1":
            # diagnostics only: one trivial launch after the idle plant step,
            # outside the timed region -- does the slow first GPU work of a step go away?
            torch.ones(1, device=dev).add_(1.0)
        if cuda:
            torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        out = run()
        if cuda:
            torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
        summ = _block_summary(out, wall, agents_per_block, world, dev)
        summ["loop_iterations"] = out.get("loop_iterations")
        per.append(summ)
        rest += out["restorations"]
    ips = [p["admm_iters_per_s"] for p in per]
    wall_tot = float(sum(p["wall_s"] for p in per))
    return {
        "control_steps": len(per),
        "admm_iters_per_s": float(sum(p["admm_iterations"] for p in per)) / wall_tot,
        "block_admm_iters_per_s": float(sum(p["block_iterations_sum"] for p in per)) / wall_tot,
        "admm_iters_per_s_median": float(np.median(ips)),
        "admm_iters_per_s_steps": ips,
        "admm_iters_per_s_spread": [float(min(ips)), float(max(ips))],
        "block_admm_iters_per_s_steps": [p["block_admm_iters_per_s"] for p in per],
        "admm_iterations_steps": [p["admm_iterations"] for p in per],
        "converged_block_fraction_steps": [p["converged_block_fraction"] for p in per],
        "block_iterations_p50_max_steps": [p["block_iterations_p50_max"] for p in per],
        "wall_s_steps": [p["wall_s"] for p in per],
        "loop_iterations_steps": [p["loop_iterations"] for p in per],
        "agent_solves_per_s": float(np.median([p["agent_solves_per_s"] for p in per])),
        "converged_solve_fraction_steps": [p["converged_solve_fraction"] for p in per],
        # the first step (cold start of every agent) in the fields the single-round leg reported
        "admm_iterations": per[0]["admm_iterations"], "converged": per[0]["converged"],
        "converged_block_fraction": per[0]["converged_block_fraction"],
        "block_iterations_p50_max": per[0]["block_iterations_p50_max"],
        **_restorations(rest, world, dev),
    }


def _warm_fleet(make_classes, run, world, dev, n_blocks=8):
    """Untimed warm-up of a coordinated leg (the contract's warmup steps): a small fleet of
    the same agent classes runs two ADMM iterations, so the timed run does not pay the
    first-use costs (caching-allocator growth, first launches, RCCL communicators) --
    measured: 0.12-0.49 s for the first C2 run vs 0.08-0.10 s for a warm one."""
    import torch
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    classes = make_classes(n_blocks)
    fl = ADMMFleet(classes, device=dev, comm="default" if world > 1 else None)
    for c in classes:
        c.native.reserve(c.n)
    run(fl)
    torch.cuda.synchronize(dev)


def _block_summary(out, wall, agents_per_block, world=1, dev=None):
    """ADMM iterations/s to consensus of a multi-block coordinated run over all ranks.  Every
    rank holds its rank-local blocks plus the blocks spanning ranks (identical copies), so
    the per-block arrays are gathered (outside the timed region) and the spanning blocks
    counted once; converged solves are summed, the wall time is the max over the ranks."""
    it = np.asarray(out["block_iterations"])
    conv = np.asarray(out["block_converged"])
    glob = np.asarray(out.get("block_is_global", np.zeros(len(it), bool)))
    iters, ok = out["iterations"], out["converged_solves"]
    if world > 1:
        import torch.distributed as dist

        parts = [None] * world
        dist.all_gather_object(parts, (it[~glob].tolist(), conv[~glob].tolist(), int(ok), float(wall), int(iters)))
        it = np.concatenate([it[glob]] + [np.asarray(p[0], np.int64) for p in parts])
        conv = np.concatenate([conv[glob]] + [np.asarray(p[1], bool) for p in parts])
        ok = sum(p[2] for p in parts)
        wall = max(p[3] for p in parts)
        iters = max(p[4] for p in parts)
    solves = int(np.sum(it)) * agents_per_block
    return {
        "admm_iterations": iters, "converged": bool(conv.all()),
        "converged_block_fraction": float(conv.mean()),
        "block_iterations_p50_max": [float(np.percentile(it, 50)), int(it.max())],
        "admm_iters_per_s": iters / wall,
        "block_admm_iters_per_s": float(it.sum()) / wall,
        "block_iterations_sum": int(it.sum()),
        "wall_s": wall,
        "agent_solves_per_s": ok / wall,
        "converged_solve_fraction": ok / max(1, solves),
    }


def _restorations(n, world, dev):
    """Calls of the feasibility restoration phase in the leg's solves, summed over the ranks
    (every leg reports it)."""
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([float(n)], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        n = int(t.item())
    return {"restorations": int(n)}


def c5_admm_bench(args, world, rank, dev):
    """C5 as the example runs it: coordinated consensus ADMM over ``--c5-blocks``
    blocks per GPU of (3 NARX zones + AHU + CCA supply)
    (`three_zone_datadriven_admm/configs/coordinator.json`: rho=1, admm_iter_max=50,
    absolute criterion primal_tol=dual_tol=0.04); each ADMM iteration = one batched
    launch per agent class + the HIP consensus/multiplier/residual kernels."""
    import torch
    import torch.distributed as dist
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.admm.fleet import ADMMFleet

    nb = args.c5_blocks
    lo, hi = bm.split_range(nb, rank, world)
    # the example's solver options are the reference IPOPT defaults
    # (`casadi_utils.py:197-206`; Room_1.json sets print_level only)
    opts = {"ipopt": {}}
    make = lambda n, off=rank * 8: bm.c5_fleet_classes(n_blocks=n, N=24, seed=20261015 + 5,  # noqa: E731
                                                      block_offset=off, solver_options=opts)
    _warm_fleet(make, lambda fl: fl.run_coordinated(1.0, admm_iter_max=2, use_relative_tolerances=False,
                                                    primal_tol=0.04, dual_tol=0.04), world, dev)
    classes = make(hi - lo, lo)
    fleet = ADMMFleet(classes, device=dev, comm="default" if world > 1 else None)
    for c in classes:
        c.native.reserve(c.n)
    loop = _closed_loop(fleet, lambda: fleet.run_coordinated(1.0, admm_iter_max=args.c5_iters,
                                                              use_relative_tolerances=False, primal_tol=0.04,
                                                              dual_tol=0.04),
                        args.admm_steps, 1800.0, 5, world, dev)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        # the first third of the GPU leg's blocks over its closed loop (5 x 50 ADMM iterations of the
        # whole fleet would take ~50 s on 16 host cores), projected by the agent ratio
        sample = bm.c5_fleet_classes(n_blocks=max(1, nb // 3), N=24, seed=20261015 + 5, solver_options=opts)
        cpu = admm_cpu_baseline_closed_loop(
            sample, lambda fl: fl.run_coordinated(1.0, admm_iter_max=args.c5_iters, use_relative_tolerances=False,
                                                  primal_tol=0.04, dual_tol=0.04),
            5 * nb, "C5 coordinated", args.admm_steps, 1800.0)
    return {
        "workload": "C5: three-zone data-driven ADMM (3 NARX zones + AHU + CCA per block), coordinated "
                    "consensus, rho=1, N=24 ts=1800, abs tol 0.04/0.04, per-block stopping",
        "scaling": "strong", "blocks_total": nb, "zones_total": 3 * nb, "agents_total": 5 * nb,
        "blocks_rank0": hi - lo if rank == 0 else None,
        **loop,
        "solver": "reference IPOPT defaults (casadi_utils.py:197-206)",
        "cpu_baseline": cpu,
    }


def admm_cpu_baseline_closed_loop(classes, run, full_agents, label, steps, ts):
    """CPU baseline of a coordinated leg over the SAME closed loop as the GPU leg (VERDICT r04
    item 5): ``steps`` control steps with the synthetic plant advanced between them
    (:func:`_closed_loop` on the host fleet: `admm/fleet.py` with `oracle/cpu_fleet.py`, every
    class's agents solved by the C IPM restatement over the class's host-compiled generated
    model, OpenMP over the host cores).  ``classes`` may be a sample of the GPU leg's fleet
    (fewer blocks): its rates are scaled to the full fleet by the agent ratio ("projected")."""
    from agentlib_mpc_amd.admm.fleet import ADMMFleet
    from oracle.cpu_fleet import CpuFleetOps

    ops = CpuFleetOps(ipopt=dict(solver_settings_ns.oracle))
    fleet = ADMMFleet(classes, device="cpu", ops=ops)
    n_sample = sum(c.n for c in classes)
    t0 = time.perf_counter()
    loop = _closed_loop(fleet, lambda: run(fleet), steps, ts, 5, 1, "cpu")
    dt = time.perf_counter() - t0
    scale = n_sample / full_agents
    unit = "ADMM iters/s" if n_sample == full_agents else "ADMM iters/s (GPU leg's fleet, projected)"
    return {"value": loop["admm_iters_per_s"] * scale, "unit": unit,
            "block_admm_iters_per_s": loop["block_admm_iters_per_s"] * scale,
            "admm_iters_per_s_steps": [v * scale for v in loop["admm_iters_per_s_steps"]],
            "admm_iterations_steps": loop["admm_iterations_steps"],
            "cores": ops.threads, "kind": "port",
            "sample": f"{label}: the GPU leg's closed loop ({loop['control_steps']} control steps, plant advanced "
                      f"between them), {sum(loop['admm_iterations_steps'])} ADMM iterations over a {n_sample}-agent "
                      f"sample fleet in {dt:.1f} s, x {n_sample}/{full_agents} agents; solves by "
                      f"oracle/c/ipm_oracle.c on host-compiled generated models, same IPOPT settings"}


def admm_cpu_baseline(classes, run, full_agents, label, min_seconds=8.0):
    """The same ADMM driver (`admm/fleet.py`) on the host: every class's agents solved by
    the C IPM restatement over the class's generated model compiled for the host
    (`oracle/c/gen_model.cpp`, OpenMP over the host cores), the ADMM arithmetic in numpy
    (`oracle/cpu_fleet.py`).  Run on the GPU leg's whole fleet (``classes``; a smaller
    sample is scaled to it by the agent ratio and labelled "projected").  The C4 leg (LocalADMM,
    one round of a fixed iteration count, no stopping rule)."""
    from agentlib_mpc_amd.admm.fleet import ADMMFleet
    from oracle.cpu_fleet import CpuFleetOps

    ops = CpuFleetOps(ipopt=dict(solver_settings_ns.oracle))
    fleet = ADMMFleet(classes, device="cpu", ops=ops)
    n_sample = sum(c.n for c in classes)
    t0 = time.perf_counter()
    iters = 0
    rounds = 0
    while rounds == 0 or time.perf_counter() - t0 < min_seconds:
        out = run(fleet)
        iters += out["iterations"]
        rounds += 1
        if rounds >= 20:
            break
    dt = time.perf_counter() - t0
    per_s = iters / dt
    unit = "ADMM iters/s" if n_sample == full_agents else "ADMM iters/s (per-GPU fleet, projected)"
    return {"value": per_s * n_sample / full_agents, "unit": unit,
            "cores": ops.threads, "kind": "port",
            "sample": f"{label}: {rounds} round(s), {iters} ADMM iterations over a {n_sample}-agent sample fleet in "
                      f"{dt:.1f} s ({per_s:.2f} it/s), x {n_sample}/{full_agents} agents; solves by "
                      f"oracle/c/ipm_oracle.c on host-compiled generated models, same IPOPT settings"}


class _SolverNS:
    oracle: dict = {}


solver_settings_ns = _SolverNS()


def e2e_bench(args, world, rank, dev):
    """One closed-loop C3 control step END TO END through the plugin API
    (``MI355XBackend.solve_batch``, the drop-in for ``OptimizationBackend.solve`` of every
    agent): new per-agent measurements in the agents' MPCVariables -> vectorised
    marshalling -> host->device copies -> one kernel launch -> solutions and stats back ->
    first control per agent (the actuation of `modules/mpc/mpc.py:342-357`).  Warm
    started from each agent's previous optimum after the first step.  The array path
    (``solve_arrays`` on [n, .] inputs, no per-agent objects) is timed beside it."""
    import copy

    import torch
    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs

    n = args.agents
    be, cv = bm.one_room(solver_options=solver_settings(args)[0])
    vals = fleet_values(n, 20261015 + 2 + rank)
    agents = []
    for a in range(n):
        c = copy.deepcopy(cv)
        for k in ("T", "load", "T_in", "T_upper", "mDot"):
            c[k].value = float(vals[k][a])
        agents.append(c)
    rng = np.random.default_rng(7 + rank)
    steps = max(2, args.steps)
    warm = max(3, args.warmup)
    be.solve_batch(0.0, agents)  # marshal maps, code object, resident inputs
    times, kernel = [], []
    # untimed warm-up control steps first: the first calls of the device scatters and of the
    # host reader run 2-3x slower than the steady state (profiles/r03/s5/e2e_prof_native.txt)
    for k in range(1, warm + steps + 1):
        drift = rng.normal(0.0, 0.05, n)
        for a, c in enumerate(agents):  # the agents' new measurements (data broker, untimed)
            c["T"].value = float(vals["T"][a] + drift[a])
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = be.solve_batch(300.0 * k, agents)
        lo, hi = cv["mDot"].lb, cv["mDot"].ub
        u0 = np.clip(res.first_values("mDot"), lo, hi)
        if k > warm:
            times.append(time.perf_counter() - t0)
            kernel.append(res.stats[0]["t_wall_total"])
    ok = sum(1 for s_ in res.stats if s_["success"])
    # array path: [n, .] inputs straight from per-agent measurement arrays
    prob = be.problem
    t_arr = []
    for k in range(steps):
        t0 = time.perf_counter()
        p, lbw, ubw, w0 = fleet_nlp_inputs(prob, cv, {key: vals[key] for key in ("T", "load", "T_in", "T_upper", "mDot")})
        r2 = be.solve_arrays(p, lbw, ubw, w0)
        u0_arr = r2.first_values("mDot")
        t_arr.append(time.perf_counter() - t0)
    # device-resident session: only the new measurements cross PCIe, warm start stays in HBM
    from agentlib_mpc_amd.optimization_backends.fleet_session import FleetSession

    sess = FleetSession(be, agents, now=0.0)
    sess.solve()
    sess.first_values("mDot")
    for k in range(warm):
        sess.update("T", vals["T"] + rng.normal(0.0, 0.05, n))
        sess.solve()
        sess.first_values("mDot")
    t_res, ok_res = [], 0
    for k in range(1, steps + 1):
        meas = vals["T"] + rng.normal(0.0, 0.05, n)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        sess.update("T", meas)
        sess.solve()
        u_res = np.clip(sess.first_values("mDot"), cv["mDot"].lb, cv["mDot"].ub)
        t_res.append(time.perf_counter() - t0)
    ok_res = int(np.isin(sess.stats().array["status"], (0, 1)).sum())
    return {
        "workload": "C3 closed-loop step through the plugin API: MPCVariable measurements of every agent -> "
                    "solve_batch (vectorised marshalling, H2D, kernel, D2H) -> first control per agent; "
                    "resident: FleetSession (inputs and warm start resident in HBM, new measurement column "
                    "H2D -> device scatter -> kernel -> first-control column D2H)",
        "agents": n, "steps": steps,
        "ms_per_step_resident": float(np.median(t_res) * 1e3),
        "solves_per_s_resident": ok_res / float(np.median(t_res)),
        "resident_converged_fraction": ok_res / n,
        "resident_actuation_checksum": float(np.sum(u_res)),
        "ms_per_step_plugin_api": float(np.median(times) * 1e3),
        "ms_per_step_solve_and_copies": float(np.median(kernel) * 1e3),
        "ms_per_step_array_path": float(np.median(t_arr) * 1e3),
        "solves_per_s_plugin_api": ok / float(np.median(times)),
        "converged_fraction": ok / n,
        "actuation_checksum": float(np.sum(u0)) + 0.0 * float(np.sum(u0_arr)),
    }


def c1_latency(args, dev):
    """C1 single-agent latency (simple_mpc, one agent): ``backend.solve(now, current_vars)``
    end to end (marshalling + copies + kernel + results), and the kernel alone (HIP events
    on the launch stream); the C restatement of the oracle on one host core beside it."""
    import torch
    from agentlib_mpc_amd import benchmarks as bm

    solver_opts, oracle_opts = solver_settings(args)
    be, cv = bm.one_room(solver_options=solver_opts)
    for _ in range(3):
        be.reset_warm_start()
        be.solve(0.0, cv)
    e2e = []
    for _ in range(20):
        be.reset_warm_start()  # cold start each time (the reference's first solve)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r = be.solve(0.0, cv)
        e2e.append(time.perf_counter() - t0)
    prob = be.problem
    p, lbw, ubw, w0 = prob.marshal.inputs([cv], 0.0)
    native = be._native()
    T = lambda a: torch.as_tensor(a, device=dev).contiguous()  # noqa: E731
    tp, tl, tu, tw0 = T(p), T(lbw), T(ubw), T(w0)
    tw = torch.empty_like(tw0)
    stream = torch.cuda.current_stream(dev)
    ks = []
    for _ in range(20):
        tw.copy_(tw0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        native.solve(tp, tl, tu, tw, stream=stream.cuda_stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ks.append(e0.elapsed_time(e1))
    out = {"workload": "C1: examples/one_room_mpc/physical/simple_mpc.py, one agent, cold start",
           "ms_end_to_end": float(np.median(e2e) * 1e3), "ms_kernel": float(np.median(ks)),
           "iter_count": int(r.stats["iter_count"]), "return_status": r.stats["return_status"],
           "build": ("small-fleet (workspace hot part in LDS, DESIGN 2.4)" if native.small_fleet_path is not None
                     else "HBM workspace")}
    try:
        from oracle import cbuild

        cbuild.build()
        opts = dict(oracle_opts)
        tol, mi = opts.pop("tol"), opts.pop("max_iter")
        t0 = time.perf_counter()
        reps = 0
        while reps < 200 and (reps == 0 or time.perf_counter() - t0 < 1.0):
            cbuild.solve_room_fleet(p, lbw, ubw, w0, tol=tol, max_iter=mi, threads=1, **opts)
            reps += 1
        out["cpu_baseline_ms"] = (time.perf_counter() - t0) / reps * 1e3
        out["cpu_baseline"] = "oracle/c/ipm_oracle.c, 1 thread, same NLP and IPOPT settings"
    except Exception as e:  # pragma: no cover
        out["cpu_baseline_error"] = repr(e)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--agents", type=int, default=4096, help="agents per GPU")
    ap.add_argument("--solver", choices=("reference", "tight"), default="reference",
                    help="reference: the reference's IPOPT defaults; tight: --tol, no acceptable stop")
    ap.add_argument("--tol", type=float, default=1e-8, help="tolerance of --solver tight")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--admm-agents", type=int, default=16384,
                    help="C4 agents in total, split over the GPUs (0: skip)")
    ap.add_argument("--admm-iters", type=int, default=15)
    ap.add_argument("--nn-zones", type=int, default=1024, help="C5 NARX zones per GPU (0: skip)")
    # 341 blocks = 1023 zones, the block count closest to BASELINE configs[4]'s 1024 zones (342
    # would be 1026); 1024 zones are one generation of the zone kernel (4 per CU x 256 CUs), and
    # two zones past it wait for a second one: 2.53 -> 4.83 ms per zone launch, 347 -> 298 ADMM
    # it/s on the leg (profiles/r04/s11)
    ap.add_argument("--c5-blocks", type=int, default=341,
                    help="C5 ADMM blocks (3 zones+AHU+CCA) in total, split over the GPUs (0: skip)")
    ap.add_argument("--c5-iters", type=int, default=50)
    ap.add_argument("--mhe-agents", type=int, default=4096, help="MHE estimators per GPU (0: skip)")
    ap.add_argument("--c2-blocks", type=int, default=1024,
                    help="C2 4-room+AHU blocks in total (1024 = the 4096-room fleet), split over the GPUs (0: skip)")
    ap.add_argument("--admm-steps", type=int, default=5,
                    help="closed-loop control steps of the coordinated legs (C2, C5), each to the stopping rule")
    ap.add_argument("--no-e2e", action="store_true", help="skip the plugin-API end-to-end leg and C1 latency")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # BENCH_DIST_BACKEND=gloo + ranks sharing a device: rehearsal of the N>1 path on
        # a one-GPU box (the driver's multi-GPU runs use nccl = RCCL, one GPU per rank)
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        gpu = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))

    from agentlib_mpc_amd import benchmarks as bm
    from agentlib_mpc_amd.optimization_backends.problem import fleet_nlp_inputs
    from agentlib_mpc_amd.runtime.native import STATS_BYTES, stats_to_dicts

    solver_opts, oracle_opts = solver_settings(args)
    solver_settings_ns.oracle = oracle_opts
    be, cv = bm.one_room(solver_options=solver_opts)
    prob = be.problem
    n = args.agents
    vals = fleet_values(n, 20261015 + 2 + rank)
    p, lbw, ubw, w0 = fleet_nlp_inputs(prob, cv, vals)
    native = be._native()
    native.reserve(n)
    tp = torch.as_tensor(p, device=dev).contiguous()
    tl = torch.as_tensor(lbw, device=dev).contiguous()
    tu = torch.as_tensor(ubw, device=dev).contiguous()
    tw0 = torch.as_tensor(w0, device=dev).contiguous()
    tw = torch.empty_like(tw0)
    lam = torch.empty((n, prob.nlp.ng_total), dtype=torch.float64, device=dev)
    st = torch.zeros(n * STATS_BYTES, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        tw.copy_(tw0)
        native.solve(tp, tl, tu, tw, lam_g=lam, stats=st, stream=stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps

    c3s = c3_strong_bench(args, world, rank, dev) if world > 1 else None
    admm = admm_bench(args, world, rank, dev) if args.admm_agents > 0 else None
    nn = nn_bench(args, world, rank, dev) if args.nn_zones > 0 else None
    c5 = c5_admm_bench(args, world, rank, dev) if args.c5_blocks > 0 else None
    c2 = c2_admm_bench(args, world, rank, dev) if args.c2_blocks > 0 else None
    mhe = mhe_bench(args, world, rank, dev) if args.mhe_agents > 0 else None
    e2e = e2e_bench(args, world, rank, dev) if not args.no_e2e else None
    c1 = c1_latency(args, dev) if not args.no_e2e and rank == 0 else None
    stats = stats_to_dicts(st.cpu().numpy().tobytes())
    n_ok = sum(1 for s in stats if s["success"])
    arr = {"iter": np.array([s["iter_count"] for s in stats]),
           "fact": np.array([s["n_factorizations"] for s in stats]),
           "trials": np.array([s["n_trials"] for s in stats]),
           "dense": np.array([s["n_dense_stages"] for s in stats])}
    flops = flops_model(prob.gen, arr)

    t_max = torch.tensor([wall], dtype=torch.float64, device=dev)
    ok_t = torch.tensor([float(n_ok)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        dist.all_reduce(ok_t, op=dist.ReduceOp.SUM)
    wall = float(t_max.item())
    total_ok = float(ok_t.item())
    value = total_ok * args.steps / wall
    if rank == 0:
        from agentlib_mpc_amd.runtime.native import code_object_path
        traffic, traffic_src = pmc_traffic(code_object_path(prob.gen.key).name, n)
        io_bytes = n * 8 * (prob.nlp.npar + 3 * prob.nlp.nw + prob.nlp.ng_total) + n * STATS_BYTES
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded per-agent C3 parameters; see bench.py docstring)",
            "config": {
                "workload": "C3: synthetic one_room fleet, batched single-shot cold-start MPC "
                            "(collocation Legendre d=2, N=15, ts=300 s), 1 agent NLP per workgroup",
                "agents_per_gpu": n,
                "agents_total": n * world,
                "nlp": prob.nlp.nlp_dims(),
                "solver": {"setting": args.solver, **oracle_opts},
                "converged_fraction_rank0": n_ok / n,
                "statuses_rank0": {k: int(v) for k, v in zip(*np.unique([s["return_status"] for s in stats],
                                                                         return_counts=True))},
                "mean_ipm_iterations": float(arr["iter"].mean()),
                "restorations_rank0": int(sum(s_["n_restorations"] for s_ in stats)),
                "soft_restorations_rank0": int(sum(s_["n_soft_restorations"] for s_ in stats)),
                "ipm_iterations_p50_p99_max": [float(np.percentile(arr["iter"], q)) for q in (50, 99, 100)],
                "parallelism": f"agent-partitioned dp{world}",
            },
            "roofline": roofline_block(kernel_ms, io_bytes, flops, traffic, traffic_src,
                                       pmc_fp64(code_object_path(prob.gen.key).name, n, kernel_ms)),
        }
        if c3s is not None:
            out["c3_strong"] = c3s
        if admm is not None:
            out["admm"] = admm
        if nn is not None:
            out["narx"] = nn
        if c5 is not None:
            out["narx_admm"] = c5
        if c2 is not None:
            out["c2_admm"] = c2
        if mhe is not None:
            out["mhe"] = mhe
        if e2e is not None:
            out["e2e"] = e2e
        if c1 is not None:
            out["c1_latency"] = c1
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(p, lbw, ubw, w0, oracle_opts)
            except Exception as e:  # pragma: no cover
                out["cpu_baseline"] = {"error": repr(e)}
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
