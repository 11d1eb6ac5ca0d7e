# restoration accuracy after the compensated p/n residuals: trace range of case 4, then the
# restoration parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/resto_diag.py trace 4 18:40 > gpurun_out/trace_4_comp.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 120 --timeout-method thread -k "restoration" > gpurun_out/gpu_resto.log 2>&1
echo "exit $?"
