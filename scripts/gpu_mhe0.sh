# stage-0 static plan (MHE): MHE GPU parity, stage-parallel test, MHE phase profile, bench legs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipm.py -m gpu -x -q -k "mhe or stage_parallel" --timeout 200 --timeout-method thread > gpurun_out/gpu_mhe.log 2>&1 && \
MODEL=mhe_room timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_mhe.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --admm-agents 0 --c2-blocks 0 > gpurun_out/legs.json 2> gpurun_out/legs.err
echo "mhe0 exit $?"
