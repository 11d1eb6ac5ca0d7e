# hot/cold workspace split: small-fleet builds for every structure; per-structure A/B, full GPU suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small_fleet or one_room" > gpurun_out/sf_quick.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/small_fleet_ab.py > gpurun_out/small_fleet_ab.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests3.log 2>&1
echo "suite exit $?"
