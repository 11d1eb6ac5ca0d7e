# single agent: per-phase cycles of the small-fleet build (MPCX_PROFILE), host profile, C1 leg;
# register-image stage elimination in the fleet builds (MHE, C3) as variants; C5 local-solve counts
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/c5_counts.py 8 > gpurun_out/c5_counts_n8.txt 2>&1 || exit $?
WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/phases_c1_lds.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/c1_prof.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base elimreg > gpurun_out/var_elimreg_mhe.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/variants.py run base elimreg base elimreg > gpurun_out/var_elimreg_c3.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture" > gpurun_out/gpu_tests_c1.txt 2>&1
echo "exit $?"
