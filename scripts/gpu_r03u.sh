# Small-batch host update path: plugin GPU tests (both paths), C1 step breakdown, C1 latency
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_plugin_batch.py tests/test_fleet_session.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/plugin_gpu2.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/e2e_prof.py 1 > gpurun_out/e2e_prof_c1.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --admm-agents 0 --c2-blocks 0 --c5-blocks 0 --mhe-agents 0 --nn-zones 0 > gpurun_out/bench_e2e2.json 2> gpurun_out/bench_e2e2.err
echo "exit $?"
