set -o pipefail
mkdir -p gpurun_out/scan
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for z in 256 512 1024 2048; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --agents 256 --no-cpu-baseline --admm-agents 0 --nn-zones $z > gpurun_out/scan/nn_$z.json 2> gpurun_out/scan/nn_$z.err || exit 1
done
for a in 1024 2048 4096 8192; do
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --agents $a --no-cpu-baseline --admm-agents 0 --nn-zones 0 > gpurun_out/scan/c3_$a.json 2> gpurun_out/scan/c3_$a.err || exit 1
done
echo "scan done"
