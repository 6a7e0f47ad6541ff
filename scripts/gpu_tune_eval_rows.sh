#!/bin/bash
# Retune the evaluation shapes' inference convs (KITTI 375x1242, Sintel 436x1024)
# with tiles 56 / 57, then KITTI inference (all-pairs / on-the-fly) new vs old table.
set -o pipefail
OUT=gpurun_out/ter
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 300 python scripts/tune_conv.py --infer-only --merge --infer-size 375 1242 --out $OUT/conv_tuning.json > $OUT/tune_kitti.log 2>&1 || { tail -20 $OUT/tune_kitti.log; exit 1; }
timeout -k 10 300 python scripts/tune_conv.py --infer-only --merge --infer-size 436 1024 --out $OUT/conv_tuning.json > $OUT/tune_sintel.log 2>&1 || { tail -20 $OUT/tune_sintel.log; exit 1; }
grep -h "best" $OUT/tune_kitti.log $OUT/tune_sintel.log
for t in new old; do
  if [[ $t == new ]]; then cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 400 python scripts/bench_configs.py --only 4 --out $OUT/k_$t.jsonl > $OUT/k.log 2>&1 || { tail -20 $OUT/k.log; exit 1; }
  echo "[$t] $(cat $OUT/k_$t.jsonl)" | tee -a $OUT/ab.txt
done
cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json
