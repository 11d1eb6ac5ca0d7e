# r04/s4: GPU parity suite (C5 N=24 fixture pending regeneration), full bench line, C1 host profile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/s4
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 120 --timeout-method thread --deselect "tests/test_gpu_admm.py::test_gpu_three_zone_narx_fleet_matches_oracle_fixture[24]" > gpurun_out/s4/gpu_tests.txt 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/s4/bench.json 2> gpurun_out/s4/bench.err || exit $?
timeout -k 10 300 python -u scripts/c1_prof.py > gpurun_out/s4/c1_prof.txt 2>&1
echo "exit $?"
