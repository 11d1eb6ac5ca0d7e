# full GPU parity suite + the C3 and end-to-end plugin legs of the bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 300 python -u bench.py --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err
echo "exit $?"
