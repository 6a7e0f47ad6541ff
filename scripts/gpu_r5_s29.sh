#!/bin/bash
# Round 5 session 29: the Chairs training feed (FlowDataset + augmentor + DataLoader) at 4 / 6 / 8 / 12 workers.
set -o pipefail
OUT=gpurun_out/r5s29
mkdir -p $OUT
export TMPDIR=/tmp
echo "nproc $(nproc)  affinity $(python -c 'import os; print(len(os.sched_getaffinity(0)))')"
for w in 4 6 8 12; do
  timeout -k 10 300 python -u scripts/bench_dataloader.py --workers $w --batch 8 --batches 80 --engine-rate 427 >> $OUT/feed.jsonl 2> $OUT/feed_err.log || { tail -20 $OUT/feed_err.log; exit 1; }
  tail -1 $OUT/feed.jsonl
done
