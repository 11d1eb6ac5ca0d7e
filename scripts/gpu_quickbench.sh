set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --admm-agents 0 > gpurun_out/qb.json 2> gpurun_out/qb.err
echo "qb exit $?"
