# r04/s13: more than 16 agents per CU (5-8 waves per SIMD) for the C4 exchange fleet's structures
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s13
MODEL=exchange_room AGENTS=13108 timeout -k 10 300 python -u scripts/variants.py run base apc20 apc24 apc32 base > gpurun_out/s13/var_apc_room.txt 2>&1 || exit $?
MODEL=exchange_supply AGENTS=3276 timeout -k 10 300 python -u scripts/variants.py run base apc20 apc24 apc32 base > gpurun_out/s13/var_apc_supply.txt 2>&1
echo "exit $?"
