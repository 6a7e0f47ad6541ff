#!/bin/bash
# Round 5 session 30: end-of-round counters of the update-block convs at the shipped tiles, training and
# inference kernel stats + the training step's stream timeline.
set -o pipefail
OUT=gpurun_out/r5s30
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train.log; exit 1; }
find /tmp/pt -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
f=$(find /tmp/pt -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/train_kernel_trace.csv.gz
python3 scripts/trace_streams.py $OUT/train_kernel_trace.csv.gz > $OUT/train_streams.txt 2>&1 || true
head -14 $OUT/train_streams.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pi -o infer -- python3 scripts/infer_only.py --reps 20 > $OUT/prof_infer.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_infer.log; exit 1; }
find /tmp/pi -name "*kernel_stats.csv" -exec cp {} $OUT/infer_kernel_stats.csv \;
CASES="gru_zr:61:8:46:62 gru_q:61:8:46:62 convc2:68:8:46:62 head:61:8:46:62 gru_zr:61:1:55:136 gru_q:34:1:55:136 convc2:61:1:55:136 head:66:1:55:136" \
  timeout -k 10 900 bash scripts/pmc_update_conv.sh > $OUT/pmc.log 2>&1 || { echo PMC FAILED; tail -20 $OUT/pmc.log; exit 1; }
cp gpurun_out/pmc_uc/summary.txt $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
