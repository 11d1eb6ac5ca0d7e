# C5 NARX parity + quick bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -v --timeout 120 --timeout-method thread -k room_nn > gpurun_out/c5_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --admm-agents 0 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err
echo "c5 exit $?"
