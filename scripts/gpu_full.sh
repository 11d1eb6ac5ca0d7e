# full bench line (all legs) + kernel-trace stats + FETCH/WRITE PMC passes on the C3 leg
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0"
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- $B > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err
echo "full exit $?"
