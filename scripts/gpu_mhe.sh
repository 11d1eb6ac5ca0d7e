# GPU parity of the MHE backend cases (plus the rest of the IPM parity file)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -v -k "${SEL:-mhe}" --timeout 120 --timeout-method thread > gpurun_out/gpu_mhe.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_mhe.log
exit $rc
