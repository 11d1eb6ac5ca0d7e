# round record (r03, after the small-fleet build / plugin reader): PMC passes of the C3 leg,
# full GPU parity suite, smoke, default bench line, rocprofv3 kernel trace of the kernel legs,
# 2-rank gloo rehearsal; stops at a crash / time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PMC_OUT=profiles/r03/final2 bash scripts/gpu_pmc.sh || exit $?
mkdir -p gpurun_out/final2 && cp profiles/r03/final2/* gpurun_out/final2/
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "suite exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || exit $?
bash scripts/gpu_mgpu_rehearsal.sh
echo "final exit $?"
