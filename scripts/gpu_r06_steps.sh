# Round-6 measurement steps, one function per step (the profiles/r06/<step> directories name them).
# Each step runs its GPU commands under their own time limits and stops at the first failure.
# usage (on the GPU box, via gpurun):  bash scripts/gpu_r06_steps.sh <step>   e.g. s1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

pmc_calib() {  # $1 = output dir: FETCH_SIZE / WRITE_SIZE of the known-bytes kernels (scripts/fetch_calib.hip)
  local o=$1
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $o/calib_fetch -o run --output-format csv -- ./scripts/bin/fetch_calib 2 > $o/calib_fetch.out 2>&1 || return $?
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $o/calib_write -o run --output-format csv -- ./scripts/bin/fetch_calib 2 > $o/calib_write.out 2>&1 || return $?
  timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $o/calib_trace -o run --output-format csv -- ./scripts/bin/fetch_calib 2 > $o/calib_trace.out 2>&1
}

step_s1() {
  # r06/s1: the RatioMin overflow fallback A/B (C3 4096 agents, tol 1e-8 runs: working tree vs HEAD);
  # the GPU suite with the collective through the C ABI (RCCL one-rank test), the wide build's
  # bench-size oracle test; smoke; FETCH_SIZE calibration; the default bench line
  mkdir -p gpurun_out/s1
  REV=HEAD timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s1/var_c3.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s1/gpu_tests.txt 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests exit $rc"; exit $rc; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.txt 2>&1 || exit $?
  pmc_calib gpurun_out/s1 || exit $?
  timeout -k 10 900 python -u bench.py > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err
  echo "tests exit $rc, bench exit $?"
}

step_s2() {
  # r06/s2: the C2 leg's slow mode with the fleet's host moves through page-locked buffers: three
  # line runs without the CPU baselines and the MHE / e2e legs (as r05/s23), round phases logged;
  # then what PC sampling this box offers, and a host-trap PC-sample histogram of the C3 leg
  mkdir -p gpurun_out/s2
  for V in a b c; do
    MPCX_FLEET_DEBUG=1 timeout -k 10 600 python -u bench.py --mhe-agents 0 --no-e2e --no-cpu-baseline > gpurun_out/s2/line_$V.json 2> gpurun_out/s2/line_$V.err || exit $?
  done
  timeout -s KILL 60 rocprofv3 -L > gpurun_out/s2/rocprof_list.txt 2>&1
  echo "list exit $?"
  grep -i -A12 "pc.sampl\|host_trap\|stochastic" gpurun_out/s2/rocprof_list.txt > gpurun_out/s2/pcs_configs.txt 2>&1
  if grep -qi "host_trap" gpurun_out/s2/rocprof_list.txt; then
    rm -rf gpurun_out/s2/pcs
    timeout -s KILL 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d gpurun_out/s2/pcs -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 --nn-zones 0 --mhe-agents 0 > gpurun_out/s2/pcs.out 2>&1
    echo "pcs exit $?"
  fi
}

step_s3() {
  # r06/s3: PMC passes of the C3 leg on the current code object (traffic, FP64 mix, wave split);
  # a kernel trace of the C2 leg alone (per-iteration spans of its rounds: scripts/iter_trace.py);
  # phase profiles of C1 (one agent, small-fleet build) and the C3 fleet
  mkdir -p gpurun_out/s3/pmc
  PMC_OUT=gpurun_out/s3/pmc bash scripts/gpu_pmc.sh || exit $?
  rm -rf gpurun_out/s3/prof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s3/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 > gpurun_out/s3/c2.json 2> gpurun_out/s3/c2.err || exit $?
  python scripts/iter_trace.py gpurun_out/s3/prof_c2 5 > gpurun_out/s3/c2_iterations.txt 2>&1
  WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s3/phases_c1_lds.txt 2>&1 || exit $?
  AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s3/phases_c3.txt 2>&1
  echo "s3 exit $?"
}

step_s4() {
  # r06/s4: no load waited for inside a branch on the hot path (acc_grad / acc_jtl unconditional,
  # the element classes from one LDS word per lane, kCIJ read with the image): A/B against HEAD on
  # the C3 fleet, C1 (small-fleet build), the C4 room fleet (13108), MHE (4096) and the C2 air handler
  # (1024); then the GPU suite, smoke and the default bench line
  mkdir -p gpurun_out/s4
  REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s4/var_c3.txt 2>&1 || exit $?
  REV=$REV AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_rev48 lds_base lds_rev48 > gpurun_out/s4/var_c1.txt 2>&1 || exit $?
  MODEL=exchange_room AGENTS=13108 REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s4/var_c4room.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s4/var_mhe.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 REV=$REV timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s4/var_ahu.txt 2>&1 || exit $?
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s4/gpu_tests.txt 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests exit $rc"; exit $rc; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s4/smoke.txt 2>&1 || exit $?
  timeout -k 10 900 python -u bench.py > gpurun_out/s4/bench.json 2> gpurun_out/s4/bench.err
  echo "tests exit $rc, bench exit $?"
}

step_s5() {
  # r06/s5: each vector phase's operands in one pinned batch (MPCX_PIN: iteration head, step recovery,
  # line search, acceptance; the solve's operator loads) against the compiler's placement (nopin) and
  # against the no-drain kernel f70845c (rev): C3, C1, the C4 room fleet, MHE, the C2 air handler
  mkdir -p gpurun_out/s5
  timeout -k 10 300 python -u scripts/variants.py run base nopin rev base nopin rev > gpurun_out/s5/var_c3.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_nopin lds_rev48 lds_base lds_nopin lds_rev48 > gpurun_out/s5/var_c1.txt 2>&1 || exit $?
  MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base nopin rev base nopin rev > gpurun_out/s5/var_c4room.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base nopin rev base nopin rev > gpurun_out/s5/var_mhe.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base nopin rev base nopin rev > gpurun_out/s5/var_ahu.txt 2>&1 || exit $?
  AGENTS=4096 timeout -k 10 400 python -u scripts/prof_phases.py > gpurun_out/s5/phases_c3.txt 2>&1
  echo "s5 exit $?"
}

step_s6() {
  # r06/s6: the vector phases' batches within a leaf phase's register budget (recover / accept: two
  # batches, variables then constraints) against the kernel of f70845c (rev) and without the iteration
  # head's pinned batch (nopin_head): C3, C1, the C4 room fleet, MHE, the C2 air handler
  mkdir -p gpurun_out/s6
  timeout -k 10 300 python -u scripts/variants.py run base nopin_head rev base nopin_head rev > gpurun_out/s6/var_c3.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_nopin_head lds_rev48 lds_base lds_nopin_head lds_rev48 > gpurun_out/s6/var_c1.txt 2>&1 || exit $?
  MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base nopin_head rev base nopin_head rev > gpurun_out/s6/var_c4room.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base nopin_head rev base nopin_head rev > gpurun_out/s6/var_mhe.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base nopin_head rev base nopin_head rev > gpurun_out/s6/var_ahu.txt 2>&1
  echo "s6 exit $?"
}

record() {
  local d=gpurun_out/$1
  # r06/s7: record on the committed kernel (two-batch vector phases, head left to the compiler): GPU
  # suite, smoke, PMC passes of the C3 leg, the default bench line, kernel-trace stats of the C3 / MHE /
  # NARX legs
  mkdir -p $d/pmc
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rfE --timeout 300 --timeout-method thread > $d/gpu_tests.txt 2>&1
  rc=$?
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && { echo "tests exit $rc"; exit $rc; }
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $d/smoke.txt 2>&1 || exit $?
  PMC_OUT=$d/pmc bash scripts/gpu_pmc.sh || exit $?
  timeout -k 10 900 python -u bench.py > $d/bench.json 2> $d/bench.err || exit $?
  rm -rf $d/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $d/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > $d/prof_bench.json 2> $d/prof.err || exit $?
  python scripts/trace_summary.py $d/prof $d/kernel_trace_summary.txt > /dev/null
  echo "tests exit $rc, record exit $?"
}

step_s9() {
  # r06/s9: the lane id masked to its range (lane_now: l & 63 -- lane-derived offsets known
  # non-negative, so loads take the SGPR-base + 32-bit offset form) against the committed kernel (rev)
  mkdir -p gpurun_out/s9
  timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s9/var_c3.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_rev48 lds_base lds_rev48 > gpurun_out/s9/var_c1.txt 2>&1 || exit $?
  MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s9/var_c4room.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s9/var_mhe.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s9/var_ahu.txt 2>&1
  echo "s9 exit $?"
}

step_s11() {
  # r06/s11: the fleet's class streams with hardware queues of their own (C ABI v15) against
  # ordinary torch streams (MPCX_FLEET_DEDICATED=0): the C2 leg (rooms + air handlers), the C5
  # leg (zones + AHU + CCA), the C4 leg; then the ADMM GPU tests and a kernel trace of the C2 leg
  mkdir -p gpurun_out/s11
  local C2="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0"
  local C5="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c2-blocks 0 --mhe-agents 0"
  local C4="--agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0"
  timeout -k 10 200 python -u -m pytest tests/test_gpu_admm.py -q -rfE --timeout 120 --timeout-method thread -k dedicated -s > gpurun_out/s11/test_dedicated.txt 2>&1 || exit $?
  for run in 1 2; do
    timeout -k 10 300 python -u bench.py $C2 > gpurun_out/s11/c2_dedicated_$run.json 2> /dev/null || exit $?
    MPCX_FLEET_DEDICATED=0 timeout -k 10 300 python -u bench.py $C2 > gpurun_out/s11/c2_torch_$run.json 2> /dev/null || exit $?
  done
  timeout -k 10 300 python -u bench.py $C5 > gpurun_out/s11/c5_dedicated.json 2> /dev/null || exit $?
  MPCX_FLEET_DEDICATED=0 timeout -k 10 300 python -u bench.py $C5 > gpurun_out/s11/c5_torch.json 2> /dev/null || exit $?
  timeout -k 10 300 python -u bench.py $C4 > gpurun_out/s11/c4_dedicated.json 2> /dev/null || exit $?
  MPCX_FLEET_DEDICATED=0 timeout -k 10 300 python -u bench.py $C4 > gpurun_out/s11/c4_torch.json 2> /dev/null || exit $?
  rm -rf gpurun_out/s11/prof_c2
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s11/prof_c2 -o run --output-format csv -- python3 bench.py $C2 > gpurun_out/s11/c2_prof.json 2> /dev/null || exit $?
  python scripts/iter_trace.py gpurun_out/s11/prof_c2 1 > gpurun_out/s11/c2_iterations.txt
  timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s11/gpu_admm_tests.txt 2>&1
  echo "s11 exit $?"
}

step_s12() {
  # r06/s12: the lead class on the caller's stream (MPCX_FLEET_LEAD_MAIN=1: two hardware queues
  # active) against both classes on class streams (default): C2, C5, C4 legs, twice each
  mkdir -p gpurun_out/s12
  local C2="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0"
  local C5="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c2-blocks 0 --mhe-agents 0"
  local C4="--agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0"
  for run in 1 2; do
    for leg in C2 C5 C4; do
      timeout -k 10 300 python -u bench.py ${!leg} > gpurun_out/s12/${leg}_default_$run.json 2> /dev/null || exit $?
      MPCX_FLEET_LEAD_MAIN=1 timeout -k 10 300 python -u bench.py ${!leg} > gpurun_out/s12/${leg}_leadmain_$run.json 2> /dev/null || exit $?
    done
  done
  rm -rf gpurun_out/s12/prof_c2
  MPCX_FLEET_LEAD_MAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s12/prof_c2 -o run --output-format csv -- python3 bench.py $C2 > gpurun_out/s12/c2_prof.json 2> /dev/null
  echo "s12 exit $?"
}

step_s13() {
  # r06/s13: the automatic lead-class placement (lead on the caller's stream unless its agents fill a
  # CU's LDS): C2, C5, C4 legs twice; the ADMM GPU tests
  mkdir -p gpurun_out/s13
  local C2="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0"
  local C5="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c2-blocks 0 --mhe-agents 0"
  local C4="--agents 64 --no-cpu-baseline --no-e2e --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0"
  for run in 1 2; do
    for leg in C2 C5 C4; do
      timeout -k 10 300 python -u bench.py ${!leg} > gpurun_out/s13/${leg}_auto_$run.json 2> /dev/null || exit $?
    done
  done
  timeout -k 10 700 python -u -m pytest tests/test_gpu_admm.py -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s13/gpu_admm_tests.txt 2>&1
  echo "s13 exit $?"
}

step_s14() {
  # r06/s14: C3 launches of 512 agents (the north-star split: 4096 rooms over 8 GPUs) and other
  # sizes, default routing, reference settings; a kernel trace of the 512-agent leg
  mkdir -p gpurun_out/s14
  local ONLY="--no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0 --steps 20 --warmup 3"
  for n in 256 512 1024 2048 4096; do
    timeout -k 10 300 python -u bench.py --agents $n $ONLY > gpurun_out/s14/c3_$n.json 2> /dev/null || exit $?
  done
  rm -rf gpurun_out/s14/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s14/prof -o run --output-format csv -- python3 bench.py --agents 512 $ONLY > gpurun_out/s14/c3_512_prof.json 2> /dev/null || exit $?
  python scripts/trace_summary.py gpurun_out/s14/prof gpurun_out/s14/kernel_trace_summary_512.txt > /dev/null
  echo "s14 exit $?"
}

step_final2() {
  # r06 final record after the fused bookkeeping (C ABI v15 header: new code objects)
  record final2 || exit $?
  bash scripts/gpu_mgpu_rehearsal.sh && mv gpurun_out/mgpu.json gpurun_out/mgpu.err gpurun_out/final2/
  echo "final2 exit $?"
}

step_final() {
  # r06 final record on the committed tree: record() + the 2-rank gloo rehearsal of bench.py's N>1 path
  record final || exit $?
  bash scripts/gpu_mgpu_rehearsal.sh && mv gpurun_out/mgpu.json gpurun_out/mgpu.err gpurun_out/final/
  echo "final exit $?"
}

step_s15() {
  # r06/s15: the line search's first trial x-part computed in recover_step (base) against the
  # committed kernel (rev)
  mkdir -p gpurun_out/s15
  timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s15/var_c3.txt 2>&1 || exit $?
  AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_rev48 lds_base lds_rev48 > gpurun_out/s15/var_c1.txt 2>&1 || exit $?
  MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s15/var_c4room.txt 2>&1 || exit $?
  MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s15/var_mhe.txt 2>&1 || exit $?
  MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base rev base rev > gpurun_out/s15/var_ahu.txt 2>&1
  echo "s15 exit $?"
}

step_repro() {
  # r06: the driver's bench command three times in separate processes (leg-to-leg reproducibility,
  # VERDICT r05 item 5)
  mkdir -p gpurun_out/repro
  for run in 1 2 3; do
    timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/repro/bench_$run.json 2> /dev/null || exit $?
  done
  echo "repro exit $?"
}

step_s16() {
  # r06/s16: the per-iteration bookkeeping fused (stats count, block expansion: one launch each for
  # all classes) against one launch per class (MPCX_FLEET_BOOK=0): ADMM GPU tests, C2 and C5 legs
  mkdir -p gpurun_out/s16
  timeout -k 10 700 python -u -m pytest tests/test_gpu_admm.py -q -rfE --timeout 300 --timeout-method thread > gpurun_out/s16/gpu_admm_tests.txt 2>&1 || exit $?
  local C2="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0"
  local C5="--agents 64 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c2-blocks 0 --mhe-agents 0"
  for run in 1 2; do
    for leg in C2 C5; do
      timeout -k 10 300 python -u bench.py ${!leg} > gpurun_out/s16/${leg}_book_$run.json 2> /dev/null || exit $?
      MPCX_FLEET_BOOK=0 timeout -k 10 300 python -u bench.py ${!leg} > gpurun_out/s16/${leg}_perclass_$run.json 2> /dev/null || exit $?
    done
  done
  echo "s16 exit $?"
}

step_s7() { record s7; }
step_s8() { record s8; }  # the record again after the non-finite-trial fix
step_s10() { record s10; }  # the record on the masked-lane kernel

fn="step_$1"
declare -F "$fn" > /dev/null || { echo "unknown step $1"; exit 2; }
"$fn"
