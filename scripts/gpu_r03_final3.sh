# round record after the hot/cold workspace split: small-fleet A/B per structure, PMC passes of
# the C3 leg, full GPU parity suite, smoke, default bench line, rocprofv3 kernel trace, 2-rank
# gloo rehearsal; stops at a crash / time limit / failing suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -q --timeout 120 --timeout-method thread -k "small_fleet or one_room" > gpurun_out/sf_quick.log 2>&1 || exit $?
timeout -k 10 400 python -u scripts/small_fleet_ab.py > gpurun_out/small_fleet_ab.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
PMC_OUT=profiles/r03/final3 bash scripts/gpu_pmc.sh || exit $?
mkdir -p gpurun_out/final3 && cp profiles/r03/final3/* gpurun_out/final3/
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || exit $?
bash scripts/gpu_mgpu_rehearsal.sh
echo "final exit $?"
