# Phase profile of the single-agent (C1-shaped) solve: HBM build vs small-fleet (LDS) build
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
AGENTS=1 timeout -k 10 200 python -u scripts/prof_phases.py > gpurun_out/phases_c1_hbm.txt 2>&1 || exit $?
AGENTS=1 WSLDS=1 timeout -k 10 200 python -u scripts/prof_phases.py > gpurun_out/phases_c1_lds.txt 2>&1 || exit $?
AGENTS=256 WSLDS=1 timeout -k 10 200 python -u scripts/prof_phases.py > gpurun_out/phases_c256_lds.txt 2>&1 || exit $?
echo done
