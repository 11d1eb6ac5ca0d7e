# fixture + ADMM GPU parity, smoke, default bench line, 2-rank gloo rehearsal of the N>1 legs
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fixtures.py tests/test_gpu_admm.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
BENCH_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --agents 1024 --admm-agents 2048 --nn-zones 256 --c5-blocks 16 --c5-iters 5 --mhe-agents 512 --c2-blocks 64 > gpurun_out/mgpu.json 2> gpurun_out/mgpu.err
echo "exit $?"
