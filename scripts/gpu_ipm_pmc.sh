# kernel iteration: IPM (+ADMM) GPU parity, C3 / NARX / MHE bench legs, FETCH/WRITE PMC passes on the C3 leg
set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --admm-agents 0 --c5-blocks 0 --c2-blocks 0 > gpurun_out/legs.json 2> gpurun_out/legs.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/fetch -o fetch --output-format csv -- $B > gpurun_out/pmc/fetch.out 2> gpurun_out/pmc/fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/write -o write --output-format csv -- $B > gpurun_out/pmc/write.out 2> gpurun_out/pmc/write.err
echo "ipm_pmc exit $?"
