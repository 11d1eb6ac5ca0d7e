# r04/s17: C2 leg variance -- the default bench line with and without the CPU baselines (which run
# OpenMP on the host before the next leg), and the C2 leg alone; then the C3 occupancy scan (s16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s17
timeout -k 10 600 python -u bench.py --no-cpu-baseline > gpurun_out/s17/bench_nocpu.json 2> gpurun_out/s17/bench_nocpu.err || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/s17/bench_default.json 2> gpurun_out/s17/bench_default.err || exit $?
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 > gpurun_out/s17/bench_c2only.json 2> gpurun_out/s17/bench_c2only.err || exit $?
bash scripts/gpu_r04_s16.sh
