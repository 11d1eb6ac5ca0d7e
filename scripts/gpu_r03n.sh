# A/B: DPP + readlane wave reductions and the lane-parallel filter test (base) vs the
# ds_bpermute butterfly (shfl) vs HEAD, C3 at 4096 / 1024 agents and MHE; IPM parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base shfl head base shfl head > gpurun_out/var_red_c3.txt 2>&1 || exit $?
AGENTS=1024 timeout -k 10 200 python -u scripts/variants.py run base shfl head base > gpurun_out/var_red_c3_1024.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base shfl head base > gpurun_out/var_red_mhe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1
echo "exit $?"
