# compile-time variants of the C3 kernel (scripts/variants.py), timed on the bench fleet
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u scripts/variants.py run ${VARIANTS:-base} > gpurun_out/variants.txt 2>&1
echo "var exit $?"
