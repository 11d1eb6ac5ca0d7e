# phase profile (MPCX_PROFILE build) + kernel-trace stats of the full bench + FETCH/WRITE PMC passes
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err
echo "profile exit $?"
