set -o pipefail
OUT=gpurun_out/r6s38
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sconv_gpu.py tests/test_sconv_train_gpu.py tests/test_model_gpu.py tests/test_export_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2; do
for v in 1 2; do
RS_SCONV_PX=$v timeout -k 10 300 python bench.py --small --steps 60 --warmup 5 --infer-reps 50 > $OUT/b$v.$r.log 2>&1 || { tail -20 $OUT/b$v.$r.log; exit 1; }
echo "px=$v run $r: $(tail -1 $OUT/b$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])')"
done
done
