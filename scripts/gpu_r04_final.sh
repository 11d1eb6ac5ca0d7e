# round-4 record: full GPU parity suite, PMC passes of the C3 leg (FETCH / WRITE / FP64 mix / issue
# split -> profiles/r04/final), smoke, default bench line (all legs + CPU baselines), rocprofv3
# kernel-trace stats of the C3 leg, 2-rank gloo rehearsal; stops at a failure / crash / time limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${DESELECT:+--deselect "$DESELECT"} > gpurun_out/final/gpu_tests.log 2>&1 || exit $?
PMC_OUT=profiles/r04/final bash scripts/gpu_pmc.sh || exit $?
mkdir -p gpurun_out/final/pmc && cp profiles/r04/final/* gpurun_out/final/pmc/
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit $?
rm -rf gpurun_out/final/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/final/prof_bench.json 2> gpurun_out/final/prof.err || exit $?
bash scripts/gpu_mgpu_rehearsal.sh
echo "final exit $?"
