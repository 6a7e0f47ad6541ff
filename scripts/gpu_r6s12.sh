set -o pipefail
OUT=gpurun_out/r6s12
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_model_gpu.py -k "small or Small" > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -3 $OUT/test.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 600 python -u scripts/tune_conv.py --small --merge --out $OUT/conv_tuning.json > $OUT/tune_small.log 2>&1 || { tail -30 $OUT/tune_small.log; exit 1; }
grep -i "8x46x62" $OUT/tune_small.log | tail -30
export RS_CONV_TUNING_FILE=$OUT/conv_tuning.json
for r in 1 2; do
for v in 0 1; do
RS_SMALL_KPAD=$v timeout -k 10 300 python bench.py --small --steps 30 --warmup 5 --no-infer > $OUT/b_small_kpad$v.$r.log 2>&1 || { tail -20 $OUT/b_small_kpad$v.$r.log; exit 1; }
echo "kpad=$v run $r: $(grep -o '"value": [0-9.]*' $OUT/b_small_kpad$v.$r.log)"
done
done
