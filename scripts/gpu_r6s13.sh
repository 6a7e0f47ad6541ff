set -o pipefail
OUT=gpurun_out/r6s13
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps -o train -- python3 bench.py --small --steps 8 --warmup 3 --no-infer > $OUT/prof_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small.log; exit 1; }
find /tmp/ps -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
f=$(find /tmp/ps -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/train_small_kernel_trace.csv.gz
python3 scripts/trace_streams.py $OUT/train_small_kernel_trace.csv.gz > $OUT/train_small_streams.txt 2>&1 || true
head -30 $OUT/train_small_streams.txt
