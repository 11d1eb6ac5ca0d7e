# per-phase cycle profile of the C3 kernel alone on its SIMD (1024 agents) and at 4096
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
MODEL=one_room AGENTS=1024 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/phases_c3_1024.txt 2>&1 || exit $?
MODEL=one_room AGENTS=4096 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/phases_c3_4096.txt 2>&1
echo "exit $?"
