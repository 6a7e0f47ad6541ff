#!/bin/bash
# Counter study of the update-block convs at the tiles the tuned table uses
# (raft_stir_amd/conv_tuning.json): training shape 8x46x62 and inference
# shape 1x55x136.  One rocprofv3 run per (shape, tile, counter pass), each
# pass within the per-block slot limits (SQ <= 8, TCC <= 4).
#   bash scripts/pmc_update_conv.sh            -> gpurun_out/pmc_uc/*.csv + summary.txt
set -o pipefail
OUT=gpurun_out/pmc_uc
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
# name:tile:batch:h:w
CASES=${CASES:-"gru_zr:31:8:46:62 gru_q:31:8:46:62 convc2:29:8:46:62 head:28:8:46:62 gru_zr:26:1:55:136 gru_q:35:1:55:136 convc2:45:1:55:136 head:26:1:55:136"}
PASSES=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
        "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum SQ_LDS_IDX_ACTIVE")
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
for c in $CASES; do
  IFS=: read name tile b h w <<< "$c"
  for i in 0 1 2; do
    tag=${name}_t${tile}_${b}x${h}x${w}_p$i
    timeout -s KILL 90 rocprofv3 --pmc ${PASSES[$i]} --output-format csv -d /tmp/pmcuc_$tag -o pmc -- \
      python3 scripts/bench_conv.py --batch $b --hw $h $w --tiles $tile --only $name --reps 5 --no-miopen \
      > $OUT/$tag.log 2>&1 || { echo "FAILED $tag"; tail -5 $OUT/$tag.log; exit 1; }
    find /tmp/pmcuc_$tag -name "*counter_collection.csv" -exec cp {} $OUT/$tag.csv \;
  done
  echo "done $name tile $tile ${b}x${h}x${w}: $(grep -h tile $OUT/${name}_t${tile}_${b}x${h}x${w}_p0.log | head -1)"
done
python3 scripts/summarize_pmc_uc.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
