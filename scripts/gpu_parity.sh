# GPU parity suite (tests marked gpu), one pytest process, per-test timeout
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_parity.log 2>&1
echo "parity exit $?"
