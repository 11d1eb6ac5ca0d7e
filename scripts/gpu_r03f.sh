# restoration line-search traces (kernel trace build vs oracle), PMC passes of the C3 leg,
# per-phase cycle profile of the C3 fleet
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/resto_diag.py trace 4 37 > gpurun_out/trace_4_37.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/resto_diag.py trace 2 44 > gpurun_out/trace_2_44.log 2>&1 || exit $?
PMC_OUT=profiles/r03/s2 bash scripts/gpu_pmc.sh || exit $?
MODEL=one_room timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/phases_c3.txt 2>&1
echo "phases exit $?"
