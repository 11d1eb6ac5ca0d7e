# r04/s12: kernel trace of the C4 (exchange ADMM, 16384 agents) and C2 legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s12
rm -rf gpurun_out/s12/prof_c4 gpurun_out/s12/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s12/prof_c4 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --c2-blocks 0 --c5-blocks 0 > gpurun_out/s12/c4.json 2> gpurun_out/s12/c4.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s12/prof_c2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c5-blocks 0 --admm-steps 1 > gpurun_out/s12/c2.json 2> gpurun_out/s12/c2.err
echo "exit $?"
