# restoration-phase parity (refined restoration steps, pruned filter) on both builds, then the
# per-truncation path comparison of the long cases; stops at a crash / time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v -rxX --timeout 300 --timeout-method thread -k "restoration or matches_oracle" > gpurun_out/resto_tests.log 2>&1
rc=$?
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -u scripts/resto_diag.py 4 60 > gpurun_out/resto_diag4.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/resto_diag.py 3 80 > gpurun_out/resto_diag3.txt 2>&1
echo "exit $?"
