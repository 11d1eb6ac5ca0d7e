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

fn="step_$1"
declare -F "$fn" > /dev/null || { echo "unknown step $1"; exit 2; }
"$fn"
