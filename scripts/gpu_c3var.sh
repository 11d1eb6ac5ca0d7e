set -o pipefail
mkdir -p gpurun_out/var
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=one_room AGENTS=4096 timeout -k 10 300 python scripts/variants.py run base lds14k lds24k lds14k_w2 lds24k_w2 > gpurun_out/var/c3_4096.log 2>&1
echo "c3var exit $?"
