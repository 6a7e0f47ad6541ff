set -o pipefail
OUT=gpurun_out/r6s17
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_norm_gpu.py tests/test_fused_encoder_gpu.py tests/test_model_gpu.py tests/test_sconv_train_gpu.py tests/test_fused_train_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps -o train -- python3 bench.py --small --steps 8 --warmup 3 --no-infer > $OUT/prof.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof.log; exit 1; }
find /tmp/ps -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
for r in 1 2; do
timeout -k 10 300 python bench.py --small --steps 60 --warmup 5 --infer-reps 30 > $OUT/b_small.$r.log 2>&1 || { tail -20 $OUT/b_small.$r.log; exit 1; }
tail -1 $OUT/b_small.$r.log
done
