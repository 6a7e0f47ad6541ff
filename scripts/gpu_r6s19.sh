set -o pipefail
OUT=gpurun_out/r6s19b
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_v3f_gpu.py tests/test_fused_train_gpu.py tests/test_model_gpu.py tests/test_fused_gpu.py -k "fp32 or f32 or v3f or F32" > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for r in 1 2; do
for v in 0 1; do
RS_V3F=$v timeout -k 10 300 python bench.py --fp32 --steps 12 --warmup 3 --infer-reps 20 > $OUT/b_fp32_v3f$v.$r.log 2>&1 || { tail -20 $OUT/b_fp32_v3f$v.$r.log; exit 1; }
echo "v3f=$v run $r: $(tail -1 $OUT/b_fp32_v3f$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])')"
done
done
