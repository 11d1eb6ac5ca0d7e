# r04/s10: the fleet's class solves on one HIP stream each (concurrent) vs one after the other:
# C4 / C2 / C5 coordinated legs, twice each; the C5 fixture tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s10
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
for i in 1 2; do
  for v in 0 1; do
    MPCX_FLEET_STREAMS=$v timeout -k 10 300 $B > gpurun_out/s10/legs_streams${v}_$i.json 2> gpurun_out/s10/legs_streams${v}_$i.err || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -q -s --timeout 300 --timeout-method thread -k "three_zone or stalled or every_block or c2" > gpurun_out/s10/gpu_admm_tests.txt 2>&1
echo "exit $?"
