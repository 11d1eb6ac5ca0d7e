# ADMM host-side bookkeeping change: ADMM GPU parity, coordinated legs, full default bench line
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_admm.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --mhe-agents 0 > gpurun_out/legs.json 2> gpurun_out/legs.err && \
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "admm_host exit $?"
