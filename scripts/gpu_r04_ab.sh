# kernel A/B on one box: C3 fleet (4096 agents) current vs the r03 kernel / filter cap 32 /
# hot phases inlined; single agent (small-fleet build) current vs phases out of line / r03;
# then the C1 latency and plugin legs of bench.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# (C3 A/B done: profiles/r04/ab_c3.txt)
AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_noinl lds_base lds_noinl > gpurun_out/ab_c1.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err

timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/c1_prof.txt 2>&1

echo "exit $?"
