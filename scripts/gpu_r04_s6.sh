# r04/s6: C1 host split, MHE per-phase cycles (4096 estimators)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s6
timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s6/c1_split.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 600 python -u scripts/prof_phases.py > gpurun_out/s6/phases_mhe.txt 2>&1
echo "exit $?"
