set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --admm-agents 0 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err && \
MODEL=room_nn AGENTS=1024 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_c5.txt 2>&1
echo "c5prof exit $?"
