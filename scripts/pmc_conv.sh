#!/bin/bash
# Counter study of the update-block conv tiles (run on the GPU box via gpurun).
#   TILES="7 10" SHAPES="gru_zr head" bash scripts/pmc_conv.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TILES=${TILES:-"7 10"}
SHAPES=${SHAPES:-"gru_zr"}
rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1 || true
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmc_$tag -o pmc -- \
    python3 scripts/bench_conv.py --batch 8 --hw 46 62 --tiles ${TILES} --only ${SHAPES} --reps 5 --no-miopen \
    > gpurun_out/pmc/$tag.log 2>&1 || return $?
  find /tmp/pmc_$tag -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc/$tag.csv \;
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run b TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum && \
run c SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM
