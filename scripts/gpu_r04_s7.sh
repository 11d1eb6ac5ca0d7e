# r04/s7: twisted state chain -- A/B against the one-sided chain (MHE, C5 zone, RNGRoom fleets), GPU parity suite
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s7
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s7/gpu_tests.txt 2>&1 || exit $?
for m in mhe_room room_nn rng_room_mpc; do
  MODEL=$m timeout -k 10 300 python -u scripts/variants.py run base chain_seq base chain_seq > gpurun_out/s7/var_chain_$m.txt 2>&1 || exit $?
done
echo "exit 0"
