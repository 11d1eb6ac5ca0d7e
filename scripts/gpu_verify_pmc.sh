# parity tests + smoke + bench + kernel-trace summary, then FETCH/WRITE PMC passes (each its own run)
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_round.sh && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err
echo "verify exit $?"
