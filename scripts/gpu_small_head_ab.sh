#!/bin/bash
# RAFT-small bf16 inference convs padded for the weight-streaming tiles (head K
# 96 -> 128, GRU-q segments to 64-multiples): tests, retune of the small / STIR
# tables, same-box A/B of the padding switches (scripts/ab_small_head.py).
set -o pipefail
OUT=gpurun_out/s52
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_model_gpu.py tests/test_export_gpu.py tests/test_fused_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
T="timeout -k 10 600 python scripts/tune_conv.py --merge --out $OUT/conv_tuning.json"
$T --small --infer-only --show "3x3|4" > $OUT/tune_small.log 2>&1 || { tail -20 $OUT/tune_small.log; exit 1; }
$T --small --infer-only --infer-size 512 640 > $OUT/tune_stir.log 2>&1 || { tail -20 $OUT/tune_stir.log; exit 1; }
grep -h "3x3|4" $OUT/tune_small.log $OUT/tune_stir.log
cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json
for r in 1 2; do for q in 1 0; do
  timeout -k 10 300 python scripts/ab_small_head.py --qpad $q -- --small --graph --reps 50 > $OUT/i.log 2>&1 || { tail -20 $OUT/i.log; exit 1; }
  timeout -k 10 300 python scripts/ab_small_head.py --qpad $q --stir -- --bf16 --reps 50 > $OUT/s.log 2>&1 || { tail -20 $OUT/s.log; exit 1; }
  echo "[qpad $q] $(tail -1 $OUT/i.log) | $(tail -1 $OUT/s.log)" | tee -a $OUT/ab.txt
done; done
