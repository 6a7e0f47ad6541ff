#!/bin/bash
# Round 5 session 5: fixed cost vs per-chunk cost of the update-block conv tiles (K sweep, batch sweep).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5s5
mkdir -p $OUT
for b in 4 8 16; do
timeout -k 10 300 python -u scripts/bench_conv.py --batch $b --hw 46 62 --reps 20 --no-miopen \
  --ksweep 64 128 256 384 768 --tiles 53 60 61 > $OUT/ksweep_b$b.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/ksweep_b$b.log; exit 1; }
echo "batch $b"; cat $OUT/ksweep_b$b.log
done
