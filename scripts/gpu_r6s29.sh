set -o pipefail
OUT=gpurun_out/r6s29
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pis -o infs -- python3 scripts/infer_only.py --small --graph --reps 20 > $OUT/prof_infer_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_infer_small.log; exit 1; }
find /tmp/pis -name "*kernel_stats.csv" -exec cp {} $OUT/infer_small_kernel_stats.csv \;
tail -1 $OUT/prof_infer_small.log
