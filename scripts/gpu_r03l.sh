# C5 N=8 divergence diagnostic (per-agent solve outcomes, iterations 10-13) and the C5 fixture tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/c5_diverge.py gpu 13 > gpurun_out/c5div_gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py -m gpu -v -s --timeout 300 --timeout-method thread -k "three_zone" > gpurun_out/gpu_c5.log 2>&1
echo "exit $?"
