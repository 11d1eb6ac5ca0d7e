# A/B: least-squares multiplier factorisation in the kernel body (base) vs HEAD on C3, MHE and
# the C5 zones; C5 fixture and restoration parity tests
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base head base head > gpurun_out/var_lsq_c3.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base head base > gpurun_out/var_lsq_mhe.txt 2>&1 || exit $?
MODEL=room_nn AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base head base > gpurun_out/var_lsq_nn.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py tests/test_gpu_ipm.py -m gpu -v -s --timeout 300 --timeout-method thread -k "three_zone or restoration or reference_defaults" > gpurun_out/gpu_sub.log 2>&1
echo "exit $?"
