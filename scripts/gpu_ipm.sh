set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1
echo "ipm exit $?"
