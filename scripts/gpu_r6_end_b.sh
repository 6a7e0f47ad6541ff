set -o pipefail
OUT=${OUT:-gpurun_out/end_b}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | tee $OUT/bench.jsonl
for a in "--small" "--fp32" "--alternate-corr" "--small --alternate-corr"; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --infer-reps 30 $a > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  tail -1 $OUT/b.log >> $OUT/bench.jsonl
done
timeout -k 10 600 python scripts/bench_configs.py --out $OUT/bench_configs.jsonl > $OUT/bench_configs.log 2>&1 || { tail -30 $OUT/bench_configs.log; exit 1; }
timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/infer_small.log 2>&1 || { tail -20 $OUT/infer_small.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_t -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train.log; exit 1; }
find /tmp/pe_t -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
f=$(find /tmp/pe_t -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/train_kernel_trace.csv.gz
python3 scripts/trace_streams.py $OUT/train_kernel_trace.csv.gz > $OUT/train_streams.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_i -o infer -- python3 scripts/infer_only.py --graph --reps 20 > $OUT/prof_infer.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_infer.log; exit 1; }
find /tmp/pe_i -name "*kernel_stats.csv" -exec cp {} $OUT/infer_kernel_stats.csv \;
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_s -o trains -- python3 bench.py --small --steps 8 --warmup 3 --no-infer > $OUT/prof_train_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train_small.log; exit 1; }
find /tmp/pe_s -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
echo done
