set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/check
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/check/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/check/smoke.log 2>&1
echo "exit $?"
