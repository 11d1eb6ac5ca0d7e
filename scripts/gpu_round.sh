set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_parity.sh
bash scripts/gpu_bench.sh
