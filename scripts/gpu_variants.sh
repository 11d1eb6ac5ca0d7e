set -o pipefail
mkdir -p gpurun_out/var
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python scripts/variants.py run > gpurun_out/var/run.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/var/fetch -o fetch --output-format csv -- python3 scripts/variants.py run base w2 inl_w2 > gpurun_out/var/fetch.log 2>&1
echo "var exit $?"
