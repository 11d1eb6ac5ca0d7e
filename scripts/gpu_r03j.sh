# occupancy scan of the C3 kernel (1024..8192 agents), PMC passes of the current code object,
# GPU parity suite, default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 1024 2048 4096 8192; do
  AGENTS=$n timeout -k 10 120 python -u scripts/variants.py run base > gpurun_out/scan_$n.txt 2>&1 || exit $?
done
PMC_OUT=profiles/r03/s3 bash scripts/gpu_pmc.sh || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "suite exit $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench exit $?"
