#!/bin/bash
# paired A/B: residual-gradient sink, host dispatch fast path (both in), headline
set -o pipefail
mkdir -p gpurun_out/s18
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for e in "X=1" "RS_RES_SINK=0" "X=1" "RS_RES_SINK=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s18/ab.log 2>&1 || { tail -20 gpurun_out/s18/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s18/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
