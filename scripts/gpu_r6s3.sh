set -o pipefail
OUT=gpurun_out/r6s3
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fused_encoder_gpu.py tests/test_norm_gpu.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.txt; exit 1; }
grep "fused encoders vs" $OUT/pytest.txt; tail -1 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_encoders.py > $OUT/enc.log 2>&1 || { tail -20 $OUT/enc.log; exit 1; }
cat $OUT/enc.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-140
RS_FUSED_ENC=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/bench0.log 2>&1 || { tail -20 $OUT/bench0.log; exit 1; }
tail -1 $OUT/bench0.log | cut -c1-140
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/bench1.log 2>&1 || { tail -20 $OUT/bench1.log; exit 1; }
tail -1 $OUT/bench1.log | cut -c1-140
