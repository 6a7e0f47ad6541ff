#!/bin/bash
# Round 5 session 23: retune the tile table with the 1x1 GEMM tile (70), A/B old vs new table on one box.
set -o pipefail
OUT=gpurun_out/r5s23
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_before.json
timeout -k 10 900 python -u scripts/tune_conv.py --merge > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "sum over" $OUT/tune.log
grep -E "best t70" $OUT/tune.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
for e in "RS_CONV_TUNING_FILE=$OUT/conv_tuning_before.json" "X=1" "RS_CONV_TUNING_FILE=$OUT/conv_tuning_before.json" "X=1"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
