set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_admm.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_admm_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --agents 256 > gpurun_out/c5admm.json 2> gpurun_out/c5admm.err
echo "c5admm exit $?"
