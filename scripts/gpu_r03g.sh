# A/B of the SGPR agent view and of inlined leaf phases (working tree vs HEAD kernel) on the
# C3 and MHE fleets, then the restoration trace range of case 4
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base head inl_gj inl_head base head > gpurun_out/var_sgpr.txt 2>&1 || exit $?
MODEL=mhe_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base head inl_gj inl_head base > gpurun_out/var_sgpr_mhe.txt 2>&1 || exit $?
timeout -k 10 800 python -u scripts/resto_diag.py trace 4 1:37 > gpurun_out/trace_4_range.log 2>&1
echo "trace exit $?"
