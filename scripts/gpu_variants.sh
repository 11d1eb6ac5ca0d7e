# A/B kernel variants on the C3 fleet (timing + FETCH_SIZE per variant)
set -o pipefail
mkdir -p gpurun_out/var
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
VARS="${VARS:-base head}"
timeout -k 10 300 python scripts/variants.py run $VARS > gpurun_out/var/run.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/var/fetch -o fetch --output-format csv -- python3 scripts/variants.py run $VARS > gpurun_out/var/fetch.log 2>&1
echo "var exit $?"
cat gpurun_out/var/run.log | grep -v -i warn
