# diagnostic: which stages take the dense path (profile build), C3 / MHE / C5 zone fleets
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases.txt 2>&1 && \
MODEL=mhe_room timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_mhe.txt 2>&1 && \
MODEL=room_nn AGENTS=1024 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_nn.txt 2>&1
echo "dense diag exit $?"
