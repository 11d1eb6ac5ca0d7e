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

fn="step_$1"
declare -F "$fn" > /dev/null || { echo "unknown step $1"; exit 2; }
"$fn"
