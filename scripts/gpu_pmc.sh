# PMC passes of the C3 leg, one counter group per run (rocprofv3 does not split passes):
# FETCH_SIZE, WRITE_SIZE (HBM/fabric traffic), the FP64 instruction mix + MFMA busy
# (FP64 utilisation) and the wave issue / wait split; summarised into $OUT.
set -o pipefail
OUT=${PMC_OUT:-profiles/r03/pmc}
mkdir -p gpurun_out/pmc "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --admm-agents 0 --nn-zones 0 --c5-blocks 0 --mhe-agents 0 --c2-blocks 0"
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc/$n -o $n --output-format csv -- $B > gpurun_out/pmc/$n.out 2> gpurun_out/pmc/$n.err
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run fp64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run issue SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SMEM && \
python scripts/pmc_summary.py "$OUT" > gpurun_out/pmc/summary.log 2>&1
echo "pmc exit $?"
