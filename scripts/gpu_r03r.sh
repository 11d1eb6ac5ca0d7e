# Native attribute reader of the plugin batch: e2e step breakdown, plugin GPU tests, bench e2e leg
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/e2e_prof.py 4096 > gpurun_out/e2e_prof_native.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_plugin_batch.py tests/test_fleet_session.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/plugin_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --admm-agents 0 --c2-blocks 0 --c5-blocks 0 --mhe-agents 0 --nn-zones 0 > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err
echo "exit $?"
