set -o pipefail
OUT=gpurun_out/r6s22
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_model_gpu.py tests/test_conv_f32_gpu.py tests/test_conv_v3f_gpu.py tests/test_export_gpu.py tests/test_train_fidelity_gpu.py tests/test_enc_f32_train_gpu.py > $OUT/test.log 2>&1 || { tail -40 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2; do
timeout -k 10 300 python bench.py --fp32 --steps 12 --warmup 3 --infer-reps 30 > $OUT/b_fp32.$r.log 2>&1 || { tail -20 $OUT/b_fp32.$r.log; exit 1; }
tail -1 $OUT/b_fp32.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"])'
done
timeout -k 10 300 python scripts/bench_configs.py --only 6 > $OUT/cfg6.log 2>&1 || { tail -5 $OUT/cfg6.log; true; }
tail -3 $OUT/cfg6.log
