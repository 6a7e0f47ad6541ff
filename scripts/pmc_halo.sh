#!/bin/bash
# Counter passes over the encoder 3x3 conv microbenchmark (halo kernel vs tiles).
set -o pipefail
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run() {  # $1 = tag, rest = counters
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d /tmp/pmch_$tag -o pmc -- \
    python3 scripts/bench_enc_halo.py --reps 3 > gpurun_out/pmc/halo_$tag.log 2>&1 || return $?
  find /tmp/pmch_$tag -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc/halo_$tag.csv \;
}
run a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE && \
run c SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM
