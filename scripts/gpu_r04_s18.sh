# r04/s18: fleet bookkeeping in one kernel per class (mpcx_stats_count): ADMM GPU tests, legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s18
timeout -k 10 900 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_fixtures.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s18/gpu_admm_tests.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s18/bench_nocpu.json 2> gpurun_out/s18/bench_nocpu.err || exit $?
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 > gpurun_out/s18/bench_c2only.json 2> gpurun_out/s18/bench_c2only.err || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/s18/bench_default.json 2> gpurun_out/s18/bench_default.err
echo "exit $?"
