# restoration-path diagnostics (truncated solves vs the oracle) + the room_nn parity cases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in 4 2 3; do
  timeout -k 10 400 python -u scripts/resto_diag.py $c 80 > gpurun_out/resto_diag_$c.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 120 --timeout-method thread -k "room_nn" > gpurun_out/gpu_nn.log 2>&1
echo "nn exit $?"
