#!/bin/bash
# Round 5 session 15: same-box A/B of this session's changes (corr backward, encoder tile 68, v3 grad sink) + stem bench.
set -o pipefail
OUT=gpurun_out/r5s15
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 200 python -u scripts/bench_stem.py > $OUT/bench_stem.log 2>&1 || { tail -20 $OUT/bench_stem.log; exit 1; }
cat $OUT/bench_stem.log
for rep in 1 2; do
for e in "X=1" "RS_AB_CORR_LIB=1" "RS_AB_T68=0" "RS_AB_SINK_V3=0"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
done
