# fused accept A/B on C3 and MHE; C5 fixture histories and the full-size C4 test
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base fused base fused > gpurun_out/var_fused_c3.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base fused base > gpurun_out/var_fused_mhe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_admm.py -m gpu -v -s --timeout 300 --timeout-method thread -k "three_zone or full_size" > gpurun_out/gpu_c5.log 2>&1
echo "exit $?"
