# r04/s15: one-wave-per-SIMD build for fleets of <= 4 agents per CU (C ABI v9): coordinated legs with
# and without it (same box), then the GPU parity suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s15
B="python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0"
for i in 1 2; do
  for v in 0 1; do
    MPCX_MID_FLEET=$v timeout -k 10 300 $B > gpurun_out/s15/legs_mid${v}_$i.json 2> gpurun_out/s15/legs_mid${v}_$i.err || exit $?
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/s15/gpu_tests.txt 2>&1
echo "exit $?"
