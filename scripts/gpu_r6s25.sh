set -o pipefail
OUT=gpurun_out/r6s25
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RS_NORM_UNROLL=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_gpu.py tests/test_norm_fused_gpu.py tests/test_fused_encoder_gpu.py > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2; do
for v in 4 8; do
RS_NORM_UNROLL=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/b$v.$r.log 2>&1 || { tail -20 $OUT/b$v.$r.log; exit 1; }
echo "unroll=$v run $r: $(tail -1 $OUT/b$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
RS_NORM_UNROLL=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_t -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train.log; exit 1; }
find /tmp/pe_t -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
