# Round-5 measurement steps, one function per step (the profiles/r05/<step> directories name them).
# Each step runs its GPU commands under their own time limits and stops at the first failure.
# usage (on the GPU box, via gpurun):  bash scripts/gpu_r05_steps.sh <step>   e.g. s1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

step_s1() {
  # r05/s1: the parity matrix over all three code objects (lds / mid / main), the 4096-agent
  # main-build C3 and C2-room tests, the ADMM suite after the single-collective change; smoke
  mkdir -p gpurun_out/s1
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s1/gpu_tests.txt 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests exit $rc"; exit $rc; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.txt 2>&1 || exit $?
  # kernel time of each code object over fleet sizes (the build choice by agents per CU)
  timeout -k 10 300 python -u scripts/build_scan.py > gpurun_out/s1/build_scan_c3.txt 2>&1 || exit $?
  MODEL=admm_room SIZES=1,64,256,512,1024,4096 timeout -k 10 300 python -u scripts/build_scan.py > gpurun_out/s1/build_scan_c2room.txt 2>&1
  echo "tests exit $rc, scan exit $?"
}

step_s2() {
  # r05/s2: kernel A/B on one box -- the working tree (barrier from the accepted trial, ratio-pair
  # step sizes, scanned scalar chain, refined reciprocals) against the previous kernel with IEEE
  # divisions (rev_ieee) and the working tree with IEEE divisions (ieee): C3 fleet (4096 agents,
  # tol 1e-8 runs) and C1 (one agent, small-fleet build); then the GPU parity suite on the new kernels
  mkdir -p gpurun_out/s2
  REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev_ieee ieee base rev_ieee ieee > gpurun_out/s2/var_c3.txt 2>&1 || exit $?
  REV=$REV AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_rev_ieee lds_ieee lds_base lds_rev_ieee lds_ieee > gpurun_out/s2/var_c1.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s2/gpu_tests.txt 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests exit $rc"; exit $rc; }
  timeout -k 10 300 python -u scripts/build_scan.py > gpurun_out/s2/build_scan_c3.txt 2>&1
  echo "tests exit $rc, scan exit $?"
}

step_s3() {
  # r05/s3: the long restoration cases with the refined reciprocals (now IEEE on 0 / inf / NaN)
  # and with IEEE divisions (MPCX_IEEE_DIV builds), the tol 1e-8 C3 A/B with iteration counts,
  # then the GPU parity suite
  mkdir -p gpurun_out/s3
  K="long_restoration"
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q -s -rfE --timeout 300 --timeout-method thread -k "$K" > gpurun_out/s3/long_resto_rcp.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  MPCX_DEFINES=MPCX_IEEE_DIV timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q -s -rfE --timeout 300 --timeout-method thread -k "$K" > gpurun_out/s3/long_resto_ieee.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 300 python -u scripts/variants.py run base ieee rev_ieee base ieee > gpurun_out/s3/var_c3_tight.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s3/gpu_tests.txt 2>&1
  echo "tests exit $?"
}

step_s4() {
  # r05/s4: which of the r05 kernel changes moves the rounding-chaotic restoration case kw1 (10
  # restoration phases at the reference settings): each diagnostic toggle alone, all of them, all
  # with IEEE divisions (main build only); then the default build
  mkdir -p gpurun_out/s4
  K="long_restoration and kw1 and main"
  for D in "" MPCX_NO_BARCACHE MPCX_RATIO_FMIN MPCX_CHAIN_SERIAL MPCX_NO_BARCACHE,MPCX_RATIO_FMIN,MPCX_CHAIN_SERIAL MPCX_IEEE_DIV,MPCX_NO_BARCACHE,MPCX_RATIO_FMIN,MPCX_CHAIN_SERIAL; do
    echo "== MPCX_DEFINES=$D" >> gpurun_out/s4/kw1.txt
    MPCX_DEFINES=$D MPCX_SMALL_FLEET=0 MPCX_MID_FLEET=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q -s --timeout 240 --timeout-method thread -k "$K" >> gpurun_out/s4/kw1.txt 2>&1
    rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  done
  # per-phase cycles of the r05 kernel: C1 (small-fleet build) and the C3 fleet
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s4/phases_c1_lds.txt 2>&1 || exit $?
  AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s4/phases_c3.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s4/gpu_tests.txt 2>&1
  echo "s4 exit $?"
}

step_s5() {
  # r05/s5: GPU parity suite on the fixed kernel (chain-scan acceptance, constant denominators),
  # the C5 fixture runs with their divergence iterations printed, then the default bench line and
  # the kernel-trace stats
  mkdir -p gpurun_out/s5
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s5/gpu_tests.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 300 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -s --timeout 240 --timeout-method thread -k "three_zone" > gpurun_out/s5/c5_fixtures.txt 2>&1
  rc2=$?; [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ] && exit $rc2
  timeout -k 10 900 python -u bench.py > gpurun_out/s5/bench.json 2> gpurun_out/s5/bench.err || exit $?
  rm -rf gpurun_out/s5/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s5/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/s5/prof_bench.json 2> gpurun_out/s5/prof.err || exit $?
  python scripts/trace_summary.py gpurun_out/s5/prof gpurun_out/s5/kernel_trace_summary.txt > /dev/null
  echo "tests exit $rc, c5 exit $rc2"
}

step_s6() {
  # r05/s6: line-search barrier as one log per lane (mantissa products) and loop-invariant
  # switching powers: kernel A/B against the committed kernel (rev) for C3 and C1; the kw1 long
  # restoration case with the inertia-correction trace on every build; then the GPU parity suite
  mkdir -p gpurun_out/s6
  REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s6/var_c3.txt 2>&1 || exit $?
  REV=$REV AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_rev lds_base lds_rev > gpurun_out/s6/var_c1.txt 2>&1 || exit $?
  MPCX_DEFINES=MPCX_TRACE_IC timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q -s -rfE --timeout 300 --timeout-method thread -k "long_restoration and kw1" > gpurun_out/s6/kw1_trace.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 600 python -u bench.py > gpurun_out/s6/bench.json 2> gpurun_out/s6/bench.err || exit $?
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s6/gpu_tests.txt 2>&1
  echo "tests exit $?"
}

step_s7() {
  # r05/s7: the kernel with the line-search barrier as one log per lane and IPOPT's constraint
  # regularisation after a failed Hessian shift (kw1 mid build: 24 shifts to 1e40 at it=46, one
  # constraint direction the Jacobian misses); GPU suite, the plugin step's host breakdown with the
  # read cache, a kernel trace of the C4 leg, the default bench line
  mkdir -p gpurun_out/s7
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s7/gpu_tests.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  timeout -k 10 300 python -u scripts/e2e_prof.py > gpurun_out/s7/e2e_prof.txt 2>&1 || exit $?
  rm -rf gpurun_out/s7/prof_c4
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s7/prof_c4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 256 --no-cpu-baseline --no-e2e --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/s7/prof_c4.json 2> gpurun_out/s7/prof_c4.err || exit $?
  python scripts/trace_summary.py gpurun_out/s7/prof_c4 gpurun_out/s7/c4_trace_summary.txt > /dev/null
  timeout -k 10 600 python -u bench.py > gpurun_out/s7/bench.json 2> gpurun_out/s7/bench.err
  echo "tests exit $rc, bench exit $?"
}

step_s8() {
  # r05/s8: the twisted chain's pivot sweeps in registers (MHE A/B against the LDS sweep), an
  # occupancy scan of the fleets that take two generations (C4 rooms, C2 rooms), the C3 phase
  # profile of the current kernel, then the GPU parity suite
  mkdir -p gpurun_out/s8
  # (the register sweep measured 8.11-8.13 ms against 8.06-8.08 ms through LDS: not kept; its
  # variant is gone from variants.py)
  MODEL=exchange_room N=13108 PER_CU=0,26,22,20,16,0 timeout -k 10 300 python -u scripts/occ_scan.py > gpurun_out/s8/occ_c4room.txt 2>&1 || exit $?
  MODEL=admm_room N=4096 PER_CU=0,24,20,16,12,0 timeout -k 10 300 python -u scripts/occ_scan.py > gpurun_out/s8/occ_c2room.txt 2>&1 || exit $?
  AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s8/phases_c3.txt 2>&1 || exit $?
  timeout -k 10 700 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s8/gpu_tests.txt 2>&1
  echo "tests exit $?"
}

step_s9() {
  # r05/s9: occupancy scan of the C4 room fleet (13108 agents, two generations at 29 per CU) with
  # the static LDS given; the C2 room code object's LDS from a kernel trace; a 512-agent C3 launch
  mkdir -p gpurun_out/s9
  MODEL=exchange_room N=13108 LDS=5632 PER_CU=0,26,22,20,16,0 timeout -k 10 300 python -u scripts/occ_scan.py > gpurun_out/s9/occ_c4room.txt 2>&1 || exit $?
  rm -rf gpurun_out/s9/prof_c2
  MODEL=admm_room N=4096 LDS=1 PER_CU=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s9/prof_c2 -o run --output-format csv -- python3 scripts/occ_scan.py > gpurun_out/s9/occ_c2_trace.txt 2>&1 || exit $?
  python scripts/trace_summary.py gpurun_out/s9/prof_c2 gpurun_out/s9/c2room_trace_summary.txt > /dev/null
  SIZES=512,1024,4096 timeout -k 10 300 python -u scripts/build_scan.py > gpurun_out/s9/build_scan_c3.txt 2>&1
  echo "s9 exit $?"
}

step_s10() {
  # r05/s10: kernel traces of the coordinated legs alone (C2: 1024 blocks, C5: 341 blocks): how
  # much of a round the GPU idles between launches (scripts/trace_gaps.py)
  mkdir -p gpurun_out/s10
  rm -rf gpurun_out/s10/prof_c2 gpurun_out/s10/prof_c5
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s10/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 > gpurun_out/s10/c2.json 2> gpurun_out/s10/c2.err || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s10/prof_c5 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c2-blocks 0 --mhe-agents 0 > gpurun_out/s10/c5.json 2> gpurun_out/s10/c5.err
  echo "s10 exit $?"
}

step_s11() {
  # r05/s11: each agent class on a hardware queue of its own (mpcx_stream_create) against plain
  # streams (MPCX_FLEET_QUEUES=0): the three ADMM legs twice each; a C2 kernel trace (queue ids);
  # the ADMM GPU tests
  mkdir -p gpurun_out/s11
  B="python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for Q in 1 0 1 0; do
    MPCX_FLEET_QUEUES=$Q timeout -k 10 300 $B > gpurun_out/s11/legs_q$Q.json.tmp 2> gpurun_out/s11/legs_q$Q.err || exit $?
    cat gpurun_out/s11/legs_q$Q.json.tmp >> gpurun_out/s11/legs_q$Q.json
  done
  rm -rf gpurun_out/s11/prof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s11/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 > gpurun_out/s11/c2.json 2> gpurun_out/s11/c2.err || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_native_abi.py -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s11/gpu_admm_tests.txt 2>&1
  echo "s11 exit $?"
}

step_s12() {
  # r05/s12: the classes' solves on the caller's stream (MPCX_FLEET_STREAMS=0: no fork / join
  # events; the plain class streams share one hardware queue anyway, s10) against one stream per
  # class: the three ADMM legs twice each
  mkdir -p gpurun_out/s12
  B="python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for S in 0 1 0 1; do
    MPCX_FLEET_STREAMS=$S timeout -k 10 300 $B > gpurun_out/s12/legs_s$S.json.tmp 2> gpurun_out/s12/legs_s$S.err || exit $?
    cat gpurun_out/s12/legs_s$S.json.tmp >> gpurun_out/s12/legs_s$S.json
  done
  echo "s12 exit $?"
}

step_s13() {
  # r05/s13: phase profiles of the current kernel: C1 (one agent, small-fleet build) and the MHE
  # fleet (4096 estimators, reference settings)
  mkdir -p gpurun_out/s13
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s13/phases_c1_lds.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s13/phases_mhe.txt 2>&1
  echo "s13 exit $?"
}

step_s14() {
  # r05/s14: a class's row moves fused into one scatter + one gather launch (C ABI v12): the ADMM
  # GPU tests (fused vs one launch per move bit for bit), the three ADMM legs fused / unfused
  # twice each; phase profiles of C1 and the MHE fleet
  mkdir -p gpurun_out/s14
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_native_abi.py -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s14/gpu_admm_tests.txt 2>&1
  rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
  B="python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for F in 1 0 1 0; do
    MPCX_FLEET_FUSED=$F timeout -k 10 300 $B > gpurun_out/s14/legs_f$F.json.tmp 2> gpurun_out/s14/legs_f$F.err || exit $?
    cat gpurun_out/s14/legs_f$F.json.tmp >> gpurun_out/s14/legs_f$F.json
  done
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s14/phases_c1_lds.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s14/phases_mhe.txt 2>&1
  echo "tests exit $rc, s14 exit $?"
}

step_s15() {
  # r05/s15: the lead class issued first, the others after its pre-solve moves (MPCX_FLEET_LEAD),
  # with the fused moves; against no lead and against unfused moves: the three ADMM legs twice
  # each; then the ADMM GPU tests
  mkdir -p gpurun_out/s15
  B="python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
  for V in L1F1 L0F1 L1F0 L1F1 L0F1 L1F0; do
    L=${V:1:1}; F=${V:3:1}
    MPCX_FLEET_LEAD=$L MPCX_FLEET_FUSED=$F timeout -k 10 300 $B > gpurun_out/s15/legs_$V.json.tmp 2> gpurun_out/s15/legs_$V.err || exit $?
    cat gpurun_out/s15/legs_$V.json.tmp >> gpurun_out/s15/legs_$V.json
  done
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s15/gpu_admm_tests.txt 2>&1
  echo "s15 exit $?"
}

step_s16() {
  # r05/s16: the full default bench line twice with the fused moves + lead class and once with
  # neither (MPCX_FLEET_LEAD=0 MPCX_FLEET_FUSED=0): the record's C2 leg fell to 741 it/s inside the
  # full line while the legs-only runs gave 1178
  mkdir -p gpurun_out/s16
  # the ADMM legs alone but WITH their CPU baselines (does the host work between legs matter?)
  timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 --agents 64 --no-e2e --nn-zones 0 --mhe-agents 0 > gpurun_out/s16/legs_cpu.json 2> gpurun_out/s16/legs_cpu.err || exit $?
  for V in L1F1 L0F0 L1F1; do
    L=${V:1:1}; F=${V:3:1}
    MPCX_FLEET_LEAD=$L MPCX_FLEET_FUSED=$F timeout -k 10 600 python -u bench.py > gpurun_out/s16/bench_$V.json.tmp 2> gpurun_out/s16/bench_$V.err || exit $?
    cat gpurun_out/s16/bench_$V.json.tmp >> gpurun_out/s16/bench_$V.json
  done
  echo "s16 exit $?"
}

step_s17() {
  # r05/s17: fused moves prepared once per fleet (no per-iteration host allocation); the full
  # default bench line normally and with the interpreter's cyclic collector off (diagnostics: is
  # the C2 leg's slowdown inside the full line the collector scanning the earlier legs' objects?);
  # the ADMM GPU tests
  mkdir -p gpurun_out/s17
  timeout -k 10 600 python -u bench.py > gpurun_out/s17/bench.json 2> gpurun_out/s17/bench.err || exit $?
  timeout -k 10 600 python -u -c "import gc, runpy, sys; gc.disable(); sys.argv = ['bench.py']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/s17/bench_nogc.json 2> gpurun_out/s17/bench_nogc.err || exit $?
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s17/gpu_admm_tests.txt 2>&1
  echo "s17 exit $?"
}

step_s18() {
  # r05/s18: which earlier leg slows the C2 leg's late steps inside the full line: the full line,
  # without the C5-zone leg, with a 64-agent C3 leg; launch sizes logged (MPCX_FLEET_DEBUG)
  mkdir -p gpurun_out/s18
  MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e > gpurun_out/s18/full.json 2> gpurun_out/s18/full.err || exit $?
  MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e --nn-zones 0 > gpurun_out/s18/nonn.json 2> gpurun_out/s18/nonn.err || exit $?
  MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e --agents 64 > gpurun_out/s18/c3small.json 2> gpurun_out/s18/c3small.err
  echo "s18 exit $?"
}

step_s19() {
  # r05/s19: the lead class's stream at high priority (its own hardware queue): three line runs
  # (no MHE / e2e legs) against two with plain streams (MPCX_FLEET_PRIO=0); launch sizes logged
  mkdir -p gpurun_out/s19
  for V in p1 p0 p1 p0 p1; do
    P=${V:1:1}
    MPCX_FLEET_PRIO=$P timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e > gpurun_out/s19/line_$V.json.tmp 2> gpurun_out/s19/line_$V.err || exit $?
    cat gpurun_out/s19/line_$V.json.tmp >> gpurun_out/s19/line_$V.json
  done
  rm -rf gpurun_out/s19/prof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s19/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 > gpurun_out/s19/c2.json 2> gpurun_out/s19/c2.err
  echo "s19 exit $?"
}

step_s20() {
  # r05/s20: where a slow C2 step's extra ~16 ms go (round prologue / loop / records, logged by
  # MPCX_FLEET_DEBUG): three line runs without the MHE / e2e legs
  mkdir -p gpurun_out/s20
  for V in a b c; do
    MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e > gpurun_out/s20/line_$V.json 2> gpurun_out/s20/line_$V.err || exit $?
  done
  echo "s20 exit $?"
}

step_s21() {
  # r05/s21: kernel trace of the line (no MHE / e2e legs) with the round phase log: what the GPU
  # does in a slow C2 round's prologue
  mkdir -p gpurun_out/s21
  rm -rf gpurun_out/s21/prof
  MPCX_FLEET_DEBUG=1 timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/s21/prof -o run --output-format csv -- python3 bench.py --mhe-agents 0 --no-e2e --no-cpu-baseline > gpurun_out/s21/line.json 2> gpurun_out/s21/line.err
  echo "s21 exit $?"
}

step_s22() {
  # r05/s22: diagnostics -- one trivial launch after each untimed plant step (MPCX_BENCH_WAKE=1)
  # in three line runs: if the C2 leg is then always fast, the slow first GPU work of a step is
  # the GPU waking from idle
  mkdir -p gpurun_out/s22
  for V in a b c; do
    MPCX_BENCH_WAKE=1 MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e --no-cpu-baseline > gpurun_out/s22/line_$V.json 2> gpurun_out/s22/line_$V.err || exit $?
  done
  echo "s22 exit $?"
}

step_s23() {
  # r05/s23: control for s22 -- the line without CPU baselines and without the wake-up launch
  mkdir -p gpurun_out/s23
  for V in a b c; do
    MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e --no-cpu-baseline > gpurun_out/s23/line_$V.json 2> gpurun_out/s23/line_$V.err || exit $?
  done
  echo "s23 exit $?"
}

step_s24() {
  # r05/s24: agents per CU of the C4 room build (MPCX_APC: 12 / 16 = default / 20 / 24 / 32, the
  # register budget following) on the 13108-room fleet
  mkdir -p gpurun_out/s24
  MODEL=exchange_room AGENTS=13108 timeout -k 10 600 python -u scripts/variants.py run base apc12 apc20 apc24 apc32 base apc20 apc24 apc32 > gpurun_out/s24/var_c4room.txt 2>&1
  echo "s24 exit $?"
}

step_s25() {
  # r05/s25: compile-flag variants of the small-fleet build on C1 (one agent): -O2, no loop
  # unrolling, a scheduler metric bias, interprocedural register allocation
  mkdir -p gpurun_out/s25
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_nounroll lds_o2 lds_maxnsa lds_ipra lds_base lds_nounroll lds_o2 lds_maxnsa lds_ipra > gpurun_out/s25/var_c1.txt 2>&1
  echo "s25 exit $?"
}

step_s26() {
  # r05/s26: the least-squares multiplier system assembled in the eliminating lane's registers
  # (assemble_reg_lsq, the default now) against the LDS-image assembly (lsq_noreg): MHE fleet and
  # C1 (one agent, small-fleet build); then the GPU parity suite on the default build.  Run at
  # 9a47260 (base = that kernel); the kernel was reverted after it (MHE 10 % slower: 1776 B scratch)
  mkdir -p gpurun_out/s26
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base lsq_noreg base lsq_noreg > gpurun_out/s26/var_mhe.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_lsq_noreg lds_base lds_lsq_noreg > gpurun_out/s26/var_c1.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s26/gpu_tests.txt 2>&1
  echo "s26 exit $?"
}

step_s27() {
  # r05/s27: the MHE twisted chain's phases (CW/CY products, pivot assembly, the swept pivots;
  # scripts/prof_phases.py CHAIN_PROF=1 on a patched copy of the kernel)
  mkdir -p gpurun_out/s27
  CHAIN_PROF=1 MODEL=mhe_room AGENTS=4096 timeout -k 10 400 python -u scripts/prof_phases.py > gpurun_out/s27/phases_mhe_chain.txt 2>&1
  echo "s27 exit $?"
}

step_s28() {
  # r05/s28: the twisted chain's pivot blocks swept on register images (bk_sweep2, readlane
  # broadcasts) against the LDS sweep (sweep_lds) on the MHE fleet; then the GPU parity suite.  Run
  # at 1bfd8f5 (base = that kernel); reverted after it (bit-identical but 29 % slower)
  mkdir -p gpurun_out/s28
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base sweep_lds base sweep_lds > gpurun_out/s28/var_mhe.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s28/gpu_tests.txt 2>&1
  echo "s28 exit $?"
}

step_s29() {
  # r05/s29: the LDS pivot sweep with its pivot values read into SGPRs (uni_f64) against f641ef4's
  # sweep (rev) on the MHE fleet.  Run at the next commit after f641ef4; reverted (2 % slower)
  mkdir -p gpurun_out/s29
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s29/var_mhe.txt 2>&1
  echo "s29 exit $?"
}

step_s30() {
  # r05/s30: the 20-agents-per-CU build of the C4 room against the default (16 per CU) over fleet
  # sizes from 1 to 6 generations of the default build on 256 CUs
  mkdir -p gpurun_out/s30
  for n in 4096 6144 8192 9216 10240 12288 13108 16384 20480 24576; do
    echo "AGENTS $n" >> gpurun_out/s30/var_c4room_sizes.txt
    MODEL=exchange_room AGENTS=$n timeout -k 10 200 python -u scripts/variants.py run base apc20 base apc20 >> gpurun_out/s30/var_c4room_sizes.txt 2>&1 || exit $?
  done
  echo "s30 exit $?"
}

step_s31() {
  # r05/s31: the GPU parity suite and smoke with the 20-agents-per-CU build (C ABI v13)
  mkdir -p gpurun_out/s31
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s31/gpu_tests.txt 2>&1 || exit $?
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s31/smoke.txt 2>&1
  echo "s31 exit $?"
}

step_rec() {
  # r05 record on the current tree ($OUT, default profiles/r05/rec): PMC passes of the C3 leg, the
  # default bench line (every leg + CPU baselines), kernel-trace stats of the C3 / MHE / NARX legs,
  # the 2-rank gloo rehearsal; TESTS=1 runs the GPU parity suite first
  OUT=${OUT:-profiles/r05/rec}
  mkdir -p gpurun_out/rec "$OUT"
  if [ "${TESTS:-0}" = 1 ]; then
    timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/rec/gpu_tests.txt 2>&1 || exit $?
    timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rec/smoke.txt 2>&1 || exit $?
  fi
  PMC_OUT=$OUT bash scripts/gpu_pmc.sh || exit $?
  mkdir -p gpurun_out/rec/pmc && cp $OUT/* gpurun_out/rec/pmc/
  timeout -k 10 900 python -u bench.py > gpurun_out/rec/bench.json 2> gpurun_out/rec/bench.err || exit $?
  rm -rf gpurun_out/rec/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rec/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/rec/prof_bench.json 2> gpurun_out/rec/prof.err || exit $?
  python scripts/trace_summary.py gpurun_out/rec/prof gpurun_out/rec/kernel_trace_summary.txt > /dev/null
  bash scripts/gpu_mgpu_rehearsal.sh > gpurun_out/rec/mgpu.txt 2>&1
  echo "rec exit $?"
}

fn="step_$1"
declare -F "$fn" > /dev/null || { echo "unknown step $1"; exit 2; }
"$fn"
