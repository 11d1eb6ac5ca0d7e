# iteration on the fleet driver: ADMM GPU parity, ADMM bench legs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_fleet_session.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_admm.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 > gpurun_out/legs_admm.json 2> gpurun_out/legs_admm.err
echo "admm iter exit $?"
