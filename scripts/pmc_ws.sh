#!/bin/bash
# Counter passes over one conv launch configuration (scripts/pmc_ws.py args in $@).
#   bash scripts/pmc_ws.sh TAG --shape 8 46 62 --k 1 5 --cin 384 --cout 256 --epi 3 --cfg 6 1 4 2 24
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/pmc_ws
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # $1 = pass name, rest = counters
  local p=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmcws_${TAG}_$p -o pmc -- \
    python3 scripts/pmc_ws.py "${ARGS[@]}" > gpurun_out/pmc_ws/${TAG}_$p.log 2>&1 || return $?
  find /tmp/pmcws_${TAG}_$p -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_ws/${TAG}_$p.csv \;
}
ARGS=("$@")
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE && \
run b SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM && \
run c TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum
