# phase profile (MPCX_PROFILE build) of the C3 fleet (and a 64-agent latency run)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases.txt 2>&1 && \
AGENTS=64 timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_64.txt 2>&1
echo "profile exit $?"
timeout -k 10 300 python scripts/c5_diag.py > gpurun_out/c5_diag.txt 2>&1
echo "c5 diag exit $?"
