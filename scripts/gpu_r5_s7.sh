#!/bin/bash
# Round 5 session 7: kernel statistics + one-step stream timeline of training, inference kernel stats,
# after the weight-streaming tiles entered the tuned table.
set -o pipefail
OUT=gpurun_out/r5s7
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o t -- python3 bench.py --steps 5 --warmup 3 --no-infer > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find /tmp/pt -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
python3 scripts/prof_categories.py $OUT/train_kernel_stats.csv 8 2>&1 | head -40 || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr -o t -- python3 bench.py --steps 1 --warmup 3 --no-infer > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
find /tmp/tr -name "*kernel_trace.csv" -exec cp {} $OUT/train_kernel_trace.csv \;
python scripts/trace_streams.py $OUT/train_kernel_trace.csv > $OUT/train_streams.txt; head -32 $OUT/train_streams.txt; gzip -f $OUT/train_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pi -o i -- python3 scripts/infer_only.py --reps 5 > $OUT/prof_infer.log 2>&1 || { tail -5 $OUT/prof_infer.log; exit 1; }
find /tmp/pi -name "*kernel_stats.csv" -exec cp {} $OUT/infer_kernel_stats.csv \;
head -12 $OUT/infer_kernel_stats.csv | cut -c1-150
