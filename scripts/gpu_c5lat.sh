set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=room_nn AGENTS=64 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_c5_64.txt 2>&1 && \
MODEL=one_room AGENTS=64 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_c3_64.txt 2>&1
echo "lat exit $?"
