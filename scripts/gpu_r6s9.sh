set -o pipefail
OUT=gpurun_out/r6s9
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "fold or corr_volume_backward" > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
tail -1 $OUT/b.log | cut -c1-150
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_t -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train.log; exit 1; }
find /tmp/pe_t -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
grep -i "fold" $OUT/train_kernel_stats.csv | cut -c1-160
timeout -k 10 600 python scripts/bench_dataloader.py --ranks 8 --workers 1 --batches 40 > $OUT/feed8x1.log 2>&1 || { tail -20 $OUT/feed8x1.log; exit 1; }
tail -1 $OUT/feed8x1.log
timeout -k 10 600 python scripts/bench_dataloader.py --ranks 1 --workers 8 --batches 60 > $OUT/feed1x8.log 2>&1 || { tail -20 $OUT/feed1x8.log; exit 1; }
tail -1 $OUT/feed1x8.log
