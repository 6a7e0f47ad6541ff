set -o pipefail
OUT=gpurun_out/r6s37
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sconv_train_gpu.py tests/test_determinism_gpu.py > $OUT/test8.log 2>&1 || { tail -30 $OUT/test8.log; exit 1; }
tail -1 $OUT/test8.log
RS_SWG_CO=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sconv_train_gpu.py > $OUT/test4.log 2>&1 || { tail -30 $OUT/test4.log; exit 1; }
tail -1 $OUT/test4.log
for r in 1 2; do
for v in 4 8; do
RS_SWG_CO=$v timeout -k 10 300 python bench.py --small --steps 60 --warmup 5 --no-infer > $OUT/b$v.$r.log 2>&1 || { tail -20 $OUT/b$v.$r.log; exit 1; }
echo "co=$v run $r: $(tail -1 $OUT/b$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
