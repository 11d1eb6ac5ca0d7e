# Small-fleet build (workspace in LDS): its parity test, C1 latency A/B (MPCX_SMALL_FLEET=0/1),
# the full GPU suite (every code object rebuilt), smoke, and the bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -v --timeout 120 --timeout-method thread -k "small_fleet or one_room" > gpurun_out/small_fleet_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  MPCX_SMALL_FLEET=$v timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --agents 256 --admm-agents 0 --c2-blocks 0 --c5-blocks 0 --mhe-agents 0 --nn-zones 0 > gpurun_out/c1_sf$v.json 2> gpurun_out/c1_sf$v.err || exit $?
  python -c "import json; d=json.load(open('gpurun_out/c1_sf$v.json')); print('small_fleet=$v', d['ms_per_step'], d['c1_latency']['ms_kernel'], d['c1_latency']['ms_end_to_end'])" >> gpurun_out/c1_ab.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_line.json 2> gpurun_out/bench.err
echo "exit $?"
