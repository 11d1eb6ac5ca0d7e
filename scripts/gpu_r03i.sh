# A/B of the inlined iteration head + derivative pass (working tree vs HEAD kernel) on C3 and
# MHE; restoration trace with inertia corrections; restoration + IPM parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base head base head > gpurun_out/var_inl_c3.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base head base > gpurun_out/var_inl_mhe.txt 2>&1 || exit $?
timeout -k 10 500 python -u scripts/resto_diag.py trace 4 17:31 > gpurun_out/trace_4_ic.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1
echo "exit $?"
