# kernel iteration: IPM + ADMM GPU parity, bench legs, compile-time variants of the C3 kernel
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --admm-agents 0 --c5-blocks 0 --c2-blocks 0 > gpurun_out/legs.json 2> gpurun_out/legs.err && \
timeout -k 10 300 python -u scripts/variants.py run base nofence nofence_ipra > gpurun_out/variants.txt 2>&1
echo "var exit $?"
