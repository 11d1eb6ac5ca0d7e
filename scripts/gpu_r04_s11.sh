# r04/s11: the C5 zone launch at one generation of agents (1024 = 256 CUs x 4) and just past it
# (1026 = 342 blocks x 3), and the coordinated C5 leg at 341 / 342 blocks
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s11
for n in 1024 1026 1023; do
  MODEL=room_nn AGENTS=$n timeout -k 10 300 python -u scripts/variants.py run base > gpurun_out/s11/var_zones_$n.txt 2>&1 || exit $?
done
for b in 341 342; do
  timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --nn-zones 0 --mhe-agents 0 --admm-agents 0 --c2-blocks 0 --c5-blocks $b > gpurun_out/s11/c5_blocks$b.json 2> gpurun_out/s11/c5_blocks$b.err || exit $?
done

timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s11/c1_split.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --mhe-agents 0 > gpurun_out/s11/bench_c1.json 2> gpurun_out/s11/bench_c1.err
echo "exit $?"
