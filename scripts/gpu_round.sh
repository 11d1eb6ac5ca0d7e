# full GPU check: parity tests, smoke, bench, rocprof kernel-trace summary
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
echo "round exit $?"
