# r04/s8: staged single-agent round trip (C ABI v8) -- C1 split / profile / leg; twisted chain (restored
# first version) A/B on MHE; GPU parity suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s8
timeout -k 10 300 python -u scripts/c1_split.py > gpurun_out/s8/c1_split.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s8/c1_prof.txt 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --admm-agents 0 --nn-zones 0 --c5-blocks 0 --c2-blocks 0 --no-cpu-baseline > gpurun_out/s8/bench_c1_mhe.json 2> gpurun_out/s8/bench_c1_mhe.err || exit $?
MODEL=mhe_room timeout -k 10 300 python -u scripts/variants.py run base chain_seq base chain_seq > gpurun_out/s8/var_chain_mhe.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s8/gpu_tests.txt 2>&1
echo "exit $?"
