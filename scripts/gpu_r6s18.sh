set -o pipefail
OUT=gpurun_out/r6s18
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf -o train -- python3 bench.py --fp32 --steps 5 --warmup 3 --no-infer > $OUT/prof_fp32.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_fp32.log; exit 1; }
find /tmp/pf -name "*kernel_stats.csv" -exec cp {} $OUT/train_fp32_kernel_stats.csv \;
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pi -o inf -- python3 scripts/infer_only.py --fp32 --graph --reps 20 > $OUT/prof_infer_fp32.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_infer_fp32.log; exit 1; }
find /tmp/pi -name "*kernel_stats.csv" -exec cp {} $OUT/infer_fp32_kernel_stats.csv \;
