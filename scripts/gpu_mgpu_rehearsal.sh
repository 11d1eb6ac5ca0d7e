# 2 ranks on the one GPU of the box over gloo: exercises bench.py's N>1 path
# (agent slices per rank, barrier + max-over-ranks timing, ADMM all-reduces)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --agents 1024 --admm-agents 2048 --nn-zones 256 --c5-blocks 16 --c5-iters 5 --mhe-agents 512 --c2-blocks 64 > gpurun_out/mgpu.json 2> gpurun_out/mgpu.err
echo "mgpu exit $?"
