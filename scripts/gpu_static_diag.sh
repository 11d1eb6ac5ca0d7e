# static vs dense stage elimination: per-case kernel statistics next to the oracle
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/static_diag.py > gpurun_out/diag_static.txt 2>&1 && \
MPCX_DEFINES=MPCX_NO_STATIC timeout -k 10 300 python -u scripts/static_diag.py > gpurun_out/diag_dense.txt 2>&1
echo "diag exit $?"
