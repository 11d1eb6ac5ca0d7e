# restoration-phase parity first, then the full GPU suite, then the kernel legs of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -v --timeout 120 --timeout-method thread -k "restoration" > gpurun_out/gpu_resto.log 2>&1
echo "resto exit $?"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "suite exit $?"
timeout -k 10 400 python -u bench.py --admm-agents 0 --c5-blocks 0 --c2-blocks 0 --no-cpu-baseline --no-e2e > gpurun_out/bench_kern.json 2> gpurun_out/bench_kern.err
echo "bench exit $?"
