# full GPU round: parity tests, smoke, bench (default), kernel-trace summary of the bench,
# FETCH_SIZE / WRITE_SIZE PMC passes on the C3 leg (each counter in its own run)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --c5-blocks 0 > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --c5-blocks 0 > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err
echo "full exit $?"
