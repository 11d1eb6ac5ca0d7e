# r04/s9: static elimination without the scheduling fences between pivot blocks (register images
# leave the scheduler free to interleave them) -- A/B on MHE, C3, C1; the staged-call GPU test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s9
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base nofence base nofence > gpurun_out/s9/var_fence_mhe.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/variants.py run base nofence base nofence > gpurun_out/s9/var_fence_c3.txt 2>&1 || exit $?
AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_nofence lds_base lds_nofence > gpurun_out/s9/var_fence_c1.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipm.py -m gpu -q --timeout 120 --timeout-method thread -k "staged or small_fleet" > gpurun_out/s9/gpu_tests.txt 2>&1
echo "exit $?"
