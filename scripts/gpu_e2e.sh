# fleet session parity + the C3 leg with the end-to-end legs (plugin API, array path, resident session, C1)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_fleet_session.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/gpu_session.log 2>&1 && \
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 > gpurun_out/e2e.json 2> gpurun_out/e2e.err
echo "e2e exit $?"
