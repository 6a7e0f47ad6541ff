set -o pipefail
OUT=gpurun_out/r6s30
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RS_SMALL_SIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_gpu.py tests/test_export_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2 3; do
for v in 0 1; do
RS_SMALL_SIDE=$v timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/inf$v.$r.log 2>&1 || { tail -5 $OUT/inf$v.$r.log; exit 1; }
echo "side=$v: $(tail -1 $OUT/inf$v.$r.log)"
done
done
