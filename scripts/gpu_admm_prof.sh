# diagnostic: kernel-trace stats of the C4 (LocalADMM) and C2 (coordinated) bench legs
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_admm -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --c5-blocks 0 --mhe-agents 0 > gpurun_out/prof_admm.json 2> gpurun_out/prof_admm.err
echo "admm prof exit $?"
