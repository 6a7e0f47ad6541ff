#!/bin/bash
# Tiles 56 / 57 (weight-streaming tiles with one / two patch rows per wave: 4x / 2x the
# blocks of tile 61 for the batch-1 grids): numerics, retune of the inference
# calls (RAFT 1088x436, RAFT-small 1088x436 and 512x640), same-box A/B of the tables.
set -o pipefail
OUT=gpurun_out/tv3r
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 400 python scripts/tune_conv.py --infer-only --merge --out $OUT/conv_tuning.json > $OUT/tune_raft.log 2>&1 || { tail -20 $OUT/tune_raft.log; exit 1; }
timeout -k 10 300 python scripts/tune_conv.py --small --infer-only --merge --out $OUT/conv_tuning.json > $OUT/tune_small.log 2>&1 || { tail -20 $OUT/tune_small.log; exit 1; }
timeout -k 10 300 python scripts/tune_conv.py --small --infer-only --merge --infer-size 512 640 --out $OUT/conv_tuning.json > $OUT/tune_stir.log 2>&1 || { tail -20 $OUT/tune_stir.log; exit 1; }
grep -h "best" $OUT/tune_raft.log $OUT/tune_small.log $OUT/tune_stir.log
for t in new old new old; do
  if [[ $t == new ]]; then cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 300 python scripts/infer_only.py --graph --reps 50 > $OUT/r.log 2>&1 || { tail -20 $OUT/r.log; exit 1; }
  timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/i.log 2>&1 || { tail -20 $OUT/i.log; exit 1; }
  timeout -k 10 300 python scripts/stir_only.py --bf16 --reps 50 > $OUT/s.log 2>&1 || { tail -20 $OUT/s.log; exit 1; }
  echo "[$t] $(tail -1 $OUT/r.log) | $(tail -1 $OUT/i.log) | $(tail -1 $OUT/s.log)" | tee -a $OUT/ab.txt
done
cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json
