# r04/s5: the eliminating lane assembles its stage image in registers (assemble_reg): A/B on MHE
# (fleet build) and C1 (small-fleet build), C1 phases / host profile / leg, GPU parity suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s5
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base asm_noreg noreg base > gpurun_out/s5/var_asmreg_mhe.txt 2>&1 || exit $?
AGENTS=1 timeout -k 10 300 python -u scripts/variants.py run lds_base lds_asm_noreg lds_noreg lds_base lds_asm_noreg lds_noreg > gpurun_out/s5/var_asmreg_c1.txt 2>&1 || exit $?
WSLDS=1 AGENTS=1 timeout -k 10 300 python -u scripts/prof_phases.py > gpurun_out/s5/phases_c1_lds.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s5/c1_prof.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/s5/bench_c1_mhe.json 2> gpurun_out/s5/bench_c1_mhe.err || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s5/gpu_tests.txt 2>&1
echo "exit $?"
