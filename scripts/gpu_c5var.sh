set -o pipefail
mkdir -p gpurun_out/var
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MODEL=room_nn AGENTS=1024 timeout -k 10 300 python scripts/variants.py run base lds20k lds14k w2 inl_w2 > gpurun_out/var/c5_1024.log 2>&1 && \
MODEL=room_nn AGENTS=128 timeout -k 10 300 python scripts/variants.py run base lds20k w2 > gpurun_out/var/c5_128.log 2>&1
echo "c5var exit $?"
