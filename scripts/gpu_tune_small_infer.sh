#!/bin/bash
# Tune RAFT-small's bf16 inference calls at the Sintel bench shape
# (1088x436), then measure bench.py --small (paired with the old table).
set -o pipefail
mkdir -p gpurun_out/tsi
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp raft_stir_amd/conv_tuning.json gpurun_out/tsi/conv_tuning.json
cp raft_stir_amd/conv_tuning.json gpurun_out/tsi/conv_tuning_old.json
timeout -k 10 300 python scripts/tune_conv.py --small --infer-only --merge --out gpurun_out/tsi/conv_tuning.json > gpurun_out/tsi/tune.log 2>&1 || { tail -20 gpurun_out/tsi/tune.log; exit 1; }
tail -n 1 gpurun_out/tsi/tune.log
for t in new old new old; do
  if [[ $t == new ]]; then cp gpurun_out/tsi/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp gpurun_out/tsi/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 300 python bench.py --small --steps 10 --warmup 5 --infer-reps 50 > gpurun_out/tsi/b.log 2>&1 || { tail -20 gpurun_out/tsi/b.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/tsi/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["inference"]["fps"])')"
done
