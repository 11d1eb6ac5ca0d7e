# Round-4 measurement steps, one function per step (the profiles/r04/<step> directories name them).
# Each step runs its GPU commands under their own time limits and stops at the first failure.
# usage (on the GPU box, via gpurun):  bash scripts/gpu_r04_steps.sh <step>   e.g. s15
# The round record itself is scripts/gpu_r04_final.sh.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

step_resto() {
  # restoration-phase parity (refined restoration steps, pruned filter) on both builds, then the
  # per-truncation path comparison of the long cases; stops at a crash / time limit
  mkdir -p gpurun_out
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v -rxX --timeout 300 --timeout-method thread -k "restoration or matches_oracle" > gpurun_out/resto_tests.log 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 300 python -u scripts/resto_diag.py 4 60 > gpurun_out/resto_diag4.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/resto_diag.py 3 80 > gpurun_out/resto_diag3.txt 2>&1
  echo "exit $?"
}

step_b() {
  # restoration / filter parity after the refinement + pruned filter (both builds)
  mkdir -p gpurun_out
  timeout -k 10 900 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v -s -rxX --timeout 300 --timeout-method thread -k "restoration or filter" > gpurun_out/resto_tests.log 2>&1
  echo "exit $?"
}

step_ab() {
  # kernel A/B on one box: C3 fleet (4096 agents) current vs the r03 kernel / filter cap 32 /
  # hot phases inlined; single agent (small-fleet build) current vs phases out of line / r03;
  # then the C1 latency and plugin legs of bench.py
  mkdir -p gpurun_out
  # (C3 A/B done: profiles/r04/ab_c3.txt)
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_noinl lds_base lds_noinl > gpurun_out/ab_c1.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err

  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/c1_prof.txt 2>&1

  echo "exit $?"
}

step_c1() {
  # single agent: per-phase cycles of the small-fleet build (MPCX_PROFILE), host profile, C1 leg;
  # register-image stage elimination in the fleet builds (MHE, C3) as variants; C5 local-solve counts
  mkdir -p gpurun_out
  timeout -k 10 300 python -u scripts/c5_counts.py 8 > gpurun_out/c5_counts_n8.txt 2>&1 || exit $?
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/phases_c1_lds.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/c1_prof.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit $?
  MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base elimreg > gpurun_out/var_elimreg_mhe.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/variants.py run base elimreg base elimreg > gpurun_out/var_elimreg_c3.txt 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture" > gpurun_out/gpu_tests_c1.txt 2>&1
  echo "exit $?"
}

step_s4() {
  # r04/s4: GPU parity suite (C5 N=24 fixture pending regeneration), full bench line, C1 host profile
  mkdir -p gpurun_out/s4
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s4/gpu_tests.txt 2>&1 || exit $?
  timeout -k 10 600 python -u bench.py > gpurun_out/s4/bench.json 2> gpurun_out/s4/bench.err || exit $?
  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s4/c1_prof.txt 2>&1
  echo "exit $?"
}

step_s5() {
  # r04/s5: the eliminating lane assembles its stage image in registers (assemble_reg): A/B on MHE
  # (fleet build) and C1 (small-fleet build), C1 phases / host profile / leg, GPU parity suite
  mkdir -p gpurun_out/s5
  MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base asm_noreg noreg base > gpurun_out/s5/var_asmreg_mhe.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_asm_noreg lds_noreg lds_base lds_asm_noreg lds_noreg > gpurun_out/s5/var_asmreg_c1.txt 2>&1 || exit $?
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s5/phases_c1_lds.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s5/c1_prof.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/s5/bench_c1_mhe.json 2> gpurun_out/s5/bench_c1_mhe.err || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s5/gpu_tests.txt 2>&1
  echo "exit $?"
}

step_s6() {
  # r04/s6: C1 host split, MHE per-phase cycles (4096 estimators)
  mkdir -p gpurun_out/s6
  timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s6/c1_split.txt 2>&1 || exit $?
  MODEL=mhe_room timeout -k 10 600 python -u scripts/prof_phases.py > gpurun_out/s6/phases_mhe.txt 2>&1
  echo "exit $?"
}

step_s7() {
  # r04/s7: twisted state chain -- A/B against the one-sided chain (MHE, C5 zone, RNGRoom fleets), GPU parity suite
  mkdir -p gpurun_out/s7
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s7/gpu_tests.txt 2>&1 || exit $?
  for m in mhe_room room_nn rng_room_mpc; do
  MODEL=$m timeout -k 10 300 python -u scripts/variants.py run base chain_seq base chain_seq > gpurun_out/s7/var_chain_$m.txt 2>&1 || exit $?
  done
  echo "exit 0"
}

step_s8() {
  # r04/s8: staged single-agent round trip (C ABI v8) -- C1 split / profile / leg; twisted chain (restored
  # first version) A/B on MHE; GPU parity suite
  mkdir -p gpurun_out/s8
  timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s8/c1_split.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s8/c1_prof.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/s8/bench_c1_mhe.json 2> gpurun_out/s8/bench_c1_mhe.err || exit $?
  MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base chain_seq base chain_seq > gpurun_out/s8/var_chain_mhe.txt 2>&1 || exit $?
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s8/gpu_tests.txt 2>&1
  echo "exit $?"
}

step_s9() {
  # r04/s9: static elimination without the scheduling fences between pivot blocks (register images
  # leave the scheduler free to interleave them) -- A/B on MHE, C3, C1; the staged-call GPU test
  mkdir -p gpurun_out/s9
  MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base nofence base nofence > gpurun_out/s9/var_fence_mhe.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/variants.py run base nofence base nofence > gpurun_out/s9/var_fence_c3.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_nofence lds_base lds_nofence > gpurun_out/s9/var_fence_c1.txt 2>&1 || exit $?
  timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q --timeout 120 --timeout-method thread -k "staged or small_fleet" > gpurun_out/s9/gpu_tests.txt 2>&1
  echo "exit $?"
}

step_s10() {
  # r04/s10: the fleet's class solves on one HIP stream each (concurrent) vs one after the other:
  # C4 / C2 / C5 coordinated legs, twice each; the C5 fixture tests
  mkdir -p gpurun_out/s10
  B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for i in 1 2; do
  for v in 0 1; do
    MPCX_FLEET_STREAMS=$v timeout -k 10 300 $B > gpurun_out/s10/legs_streams${v}_$i.json 2> gpurun_out/s10/legs_streams${v}_$i.err || exit $?
  done
  done
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -s --timeout 300 --timeout-method thread -k "three_zone or stalled or every_block or c2" > gpurun_out/s10/gpu_admm_tests.txt 2>&1
  echo "exit $?"
}

step_s11() {
  # r04/s11: the C5 zone launch at one generation of agents (1024 = 256 CUs x 4) and just past it
  # (1026 = 342 blocks x 3), and the coordinated C5 leg at 341 / 342 blocks
  mkdir -p gpurun_out/s11
  for n in 1024 1026 1023; do
  MODEL=room_nn AGENTS=$n timeout -k 10 300 python -u scripts/variants.py run base > gpurun_out/s11/var_zones_$n.txt 2>&1 || exit $?
  done
  for b in 341 342; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c2-blocks 0 --c5-blocks $b > gpurun_out/s11/c5_blocks$b.json 2> gpurun_out/s11/c5_blocks$b.err || exit $?
  done

  timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s11/c1_split.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0 > gpurun_out/s11/bench_c1.json 2> gpurun_out/s11/bench_c1.err
  echo "exit $?"
}

step_s12() {
  # r04/s12: kernel trace of the C4 (exchange ADMM, 16384 agents) and C2 legs
  mkdir -p gpurun_out/s12
  rm -rf gpurun_out/s12/prof_c4 gpurun_out/s12/prof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s12/prof_c4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/s12/c4.json 2> gpurun_out/s12/c4.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s12/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 --admm-steps 1 > gpurun_out/s12/c2.json 2> gpurun_out/s12/c2.err
  echo "exit $?"
}

step_s13() {
  # r04/s13: more than 16 agents per CU (5-8 waves per SIMD) for the C4 exchange fleet's structures
  mkdir -p gpurun_out/s13
  MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base apc20 apc24 apc32 base > gpurun_out/s13/var_apc_room.txt 2>&1 || exit $?
  MODEL=exchange_supply AGENTS=3276 timeout -k 10 300 python -u scripts/variants.py run base apc20 apc24 apc32 base > gpurun_out/s13/var_apc_supply.txt 2>&1
  echo "exit $?"
}

step_s14() {
  # r04/s14: register budget vs occupancy for the C2 structures at their fleet sizes (4096 rooms,
  # 1024 air handlers): 4 (base, 128 VGPRs) / 3 / 2 / 1 waves per SIMD
  mkdir -p gpurun_out/s14
  MODEL=admm_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base w3 w2 base > gpurun_out/s14/var_w_room4096.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base w3 w2 w1 base > gpurun_out/s14/var_w_ahu1024.txt 2>&1
  echo "exit $?"
}

step_s15() {
  # r04/s15: one-wave-per-SIMD build for fleets of <= 4 agents per CU (C ABI v9): coordinated legs with
  # and without it (same box), then the GPU parity suite
  mkdir -p gpurun_out/s15
  B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for i in 1 2; do
  for v in 0 1; do
    MPCX_MID_FLEET=$v timeout -k 10 300 $B > gpurun_out/s15/legs_mid${v}_$i.json 2> gpurun_out/s15/legs_mid${v}_$i.err || exit $?
  done
  done
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s15/gpu_tests.txt 2>&1
  echo "exit $?"
}

step_s16() {
  # r04/s16: occupancy scan of the C3 structure on the r04 kernel (1, 2, 4 waves per SIMD: 1024 /
  # 2048 / 4096 agents; the main build, the one-wave-per-SIMD build at 1024) -- the measurement the
  # lane-packing analysis rests on
  mkdir -p gpurun_out/s16
  for n in 1024 2048 4096; do
  AGENTS=$n timeout -k 10 300 python -u scripts/variants.py run base > gpurun_out/s16/occ_$n.txt 2>&1 || exit $?
  done
  AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run w1 > gpurun_out/s16/occ_1024_w1.txt 2>&1
  echo "exit $?"
}

step_s17() {
  # r04/s17: C2 leg variance -- the default bench line with and without the CPU baselines (which run
  # OpenMP on the host before the next leg), and the C2 leg alone; then the C3 occupancy scan (s16)
  mkdir -p gpurun_out/s17
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s17/bench_nocpu.json 2> gpurun_out/s17/bench_nocpu.err || exit $?
  timeout -k 10 600 python -u bench.py > gpurun_out/s17/bench_default.json 2> gpurun_out/s17/bench_default.err || exit $?
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 > gpurun_out/s17/bench_c2only.json 2> gpurun_out/s17/bench_c2only.err || exit $?
  step_s16
}

step_s18() {
  # r04/s18: fleet bookkeeping in one kernel per class (mpcx_stats_count): ADMM GPU tests, legs
  mkdir -p gpurun_out/s18
  timeout -k 10 900 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_fixtures.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s18/gpu_admm_tests.txt 2>&1 || exit $?
  timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s18/bench_nocpu.json 2> gpurun_out/s18/bench_nocpu.err || exit $?
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 > gpurun_out/s18/bench_c2only.json 2> gpurun_out/s18/bench_c2only.err || exit $?
  timeout -k 10 600 python -u bench.py > gpurun_out/s18/bench_default.json 2> gpurun_out/s18/bench_default.err
  echo "exit $?"
}

step_s19() {
  # r04/s19: single-agent result objects from the host mirrors -- plugin / fixture GPU tests, C1 leg
  mkdir -p gpurun_out/s19
  timeout -k 10 600 python -u -m pytest tests/test_plugin_batch.py tests/test_gpu_fixtures.py tests/test_gpu_ipm.py -m gpu -q --timeout 300 --timeout-method thread -k "plugin or fixture or permuted or staged or reference or c1 or one_room" > gpurun_out/s19/gpu_tests.txt 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0 > gpurun_out/s19/bench_c1.json 2> gpurun_out/s19/bench_c1.err || exit $?
  timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s19/c1_prof.txt 2>&1
  echo "exit $?"
}

step_s20() {
  # r04/s20: ADMM GPU tests and the legs after the last fleet change (finalize skip)
  mkdir -p gpurun_out/s20
  timeout -k 10 900 python -u -m pytest tests/test_gpu_admm.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s20/gpu_admm_tests.txt 2>&1 || exit $?
  timeout -k 10 600 python -u bench.py > gpurun_out/s20/bench_default.json 2> gpurun_out/s20/bench_default.err
  echo "exit $?"
}

step_s21() {
  # MHE per-phase cycles after the register-image elimination and the twisted chain
  mkdir -p gpurun_out/s21
  MODEL=mhe_room timeout -k 10 600 python -u scripts/prof_phases.py > gpurun_out/s21/phases_mhe.txt 2>&1
  echo "exit $?"
}

fn="step_$1"
declare -F "$fn" > /dev/null || { echo "unknown step $1"; exit 2; }
"$fn"
