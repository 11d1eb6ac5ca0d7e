# C3 phase profile + two runs of the bench legs (run-to-run spread of the coordinated legs)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=one_room timeout -k 10 200 python scripts/prof_phases.py > gpurun_out/phases_c3.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/legs_a.json 2> gpurun_out/legs_a.err && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/legs_b.json 2> gpurun_out/legs_b.err
echo "c3phase exit $?"
