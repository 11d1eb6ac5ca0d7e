set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BLOCKS=32 ITERS=50 TOL=1e-4 MAXIT=100 timeout -k 10 300 python scripts/c5_admm_diag.py > gpurun_out/c5diag.log 2>&1
echo "diag exit $?"
