# r04/s16: occupancy scan of the C3 structure on the r04 kernel (1, 2, 4 waves per SIMD: 1024 /
# 2048 / 4096 agents; the main build, the one-wave-per-SIMD build at 1024) -- the measurement the
# lane-packing analysis rests on
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s16
for n in 1024 2048 4096; do
  AGENTS=$n timeout -k 10 300 python -u scripts/variants.py run base > gpurun_out/s16/occ_$n.txt 2>&1 || exit $?
done
AGENTS=1024 timeout -k 10 300 python -u scripts/variants.py run w1 > gpurun_out/s16/occ_1024_w1.txt 2>&1
echo "exit $?"
