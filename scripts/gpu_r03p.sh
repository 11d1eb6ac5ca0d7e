# A/B: vector phases with every operand loaded first (base: + recover/accept inlined;
# noinl_ra: recover/accept out of line) vs HEAD, C3 at 4096 / 1024 agents and MHE; IPM parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/variants.py run base head noinl_ra base head noinl_ra > gpurun_out/var_ld_c3.txt 2>&1 || exit $?
AGENTS=1024 timeout -k 10 200 python -u scripts/variants.py run base head noinl_ra base > gpurun_out/var_ld_c3_1024.txt 2>&1 || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base head noinl_ra base > gpurun_out/var_ld_mhe.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_ipm.log 2>&1
echo "exit $?"
