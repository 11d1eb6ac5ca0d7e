# chain-pivot change: IPM + ADMM GPU parity, MHE / NARX phase profiles, bench legs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py tests/test_gpu_admm.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1 && \
MODEL=mhe_room timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_mhe.txt 2>&1 && \
MODEL=room_nn AGENTS=1024 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_nn.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/legs.json 2> gpurun_out/legs.err
echo "chain exit $?"
