# diagnostic: per-phase cycle profile (MPCX_PROFILE build) of the MHE and the 2-state zone MPC fleets
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=mhe_room timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_mhe.txt 2>&1 && \
MODEL=rng_room_mpc timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_rng.txt 2>&1
echo "phases exit $?"
