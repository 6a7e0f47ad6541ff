#!/bin/bash
# Round 5 session 32: encoder conv weight gradients on the deferred-gradient stream (A/B, same box).
set -o pipefail
OUT=gpurun_out/r5s32
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for rep in 1 2 3; do
for e in "X=1" "RS_AB_DEFER_ENC=1"; do
  env $e timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
