#!/bin/bash
# Retune RAFT-small's batch-1 inference convs (Sintel 436x1088 and the STIR
# tracker's 512x640) now that the weight-streaming tiles 60-68 exist, then a
# same-box A/B of the new table against the old one (RAFT-small inference FPS,
# STIR served latency, and the headline as a guard).
set -o pipefail
OUT=gpurun_out/tsv3
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 300 python scripts/tune_conv.py --small --infer-only --merge --out $OUT/conv_tuning.json > $OUT/tune_sintel.log 2>&1 || { tail -20 $OUT/tune_sintel.log; exit 1; }
timeout -k 10 300 python scripts/tune_conv.py --small --infer-only --merge --infer-size 512 640 --out $OUT/conv_tuning.json > $OUT/tune_stir.log 2>&1 || { tail -20 $OUT/tune_stir.log; exit 1; }
grep -h "best" $OUT/tune_sintel.log $OUT/tune_stir.log
for t in new old new old; do
  if [[ $t == new ]]; then cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/i.log 2>&1 || { tail -20 $OUT/i.log; exit 1; }
  timeout -k 10 300 python scripts/stir_only.py --bf16 --reps 50 > $OUT/s.log 2>&1 || { tail -20 $OUT/s.log; exit 1; }
  echo "[$t] $(tail -1 $OUT/i.log) | $(tail -1 $OUT/s.log)" | tee -a $OUT/ab.txt
done
cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json
