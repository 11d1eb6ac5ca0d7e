set -o pipefail
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests/test_gpu_ipm.py -x -q > gpurun_out/gpu1.log 2>&1
echo "exit $?" >> gpurun_out/gpu1.log
