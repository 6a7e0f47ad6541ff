#!/bin/bash
# Retune the training-shape conv calls with tiles 56 / 57 among the candidates,
# then a same-box A/B of the new table against the old one (headline bench).
set -o pipefail
OUT=gpurun_out/ttr
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 600 python scripts/tune_conv.py --merge --out $OUT/conv_tuning.json > $OUT/tune_train.log 2>&1 || { tail -20 $OUT/tune_train.log; exit 1; }
grep -h "best" $OUT/tune_train.log
for t in new old new old; do
  if [[ $t == new ]]; then cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 400 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  echo "[$t] $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("inference") or {}).get("fps"))')" | tee -a $OUT/ab.txt
done
cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json
