set -o pipefail
OUT=gpurun_out/r6s14d
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in 64; do
RS_WIDE_GEO=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pw$v -o train -- python3 bench.py --small --steps 8 --warmup 3 --no-infer > $OUT/prof_wide$v.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_wide$v.log; exit 1; }
find /tmp/pw$v -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats_wide$v.csv \;
done
