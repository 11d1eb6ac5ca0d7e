# r04/s14: register budget vs occupancy for the C2 structures at their fleet sizes (4096 rooms,
# 1024 air handlers): 4 (base, 128 VGPRs) / 3 / 2 / 1 waves per SIMD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s14
MODEL=admm_room AGENTS=4096 timeout -k 10 300 python -u scripts/variants.py run base w3 w2 base > gpurun_out/s14/var_w_room4096.txt 2>&1 || exit $?
MODEL=admm_ahu AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run base w3 w2 w1 base > gpurun_out/s14/var_w_ahu1024.txt 2>&1
echo "exit $?"
