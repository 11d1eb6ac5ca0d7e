# diagnostic: per-phase cycle profile (MPCX_PROFILE build) of the C3 fleet and the C5 zone
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases.txt 2>&1 && \
MODEL=room_nn AGENTS=1024 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_nn.txt 2>&1
echo "phases exit $?"
