# round record: FETCH/WRITE PMC passes of the C3 leg (summarised first, so the bench line
# carries the traffic of this code object), full GPU parity suite, smoke, default bench line
# (all legs + CPU baselines), rocprofv3 kernel-trace stats of the C3 leg
set -o pipefail
OUT=${PMC_OUT:-profiles/r02/s12}
mkdir -p gpurun_out/pmc "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- $B > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err && \
python scripts/pmc_summary.py "$OUT" > gpurun_out/pmc/summary.log 2>&1 && cp "$OUT/pmc_traffic_c3.json" gpurun_out/pmc_traffic_c3.json && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err
echo "final exit $?"
