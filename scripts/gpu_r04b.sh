# restoration / filter parity after the refinement + pruned filter (both builds)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ipm.py -m gpu -v -s -rxX --timeout 300 --timeout-method thread -k "restoration or filter" > gpurun_out/resto_tests.log 2>&1
echo "exit $?"
