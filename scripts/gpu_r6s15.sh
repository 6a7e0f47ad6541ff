set -o pipefail
OUT=gpurun_out/r6s15
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py tests/test_determinism_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for r in 1 2; do
for v in 0 1; do
RS_EARLY_CORR_BWD=$v timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-infer > $OUT/b_early$v.$r.log 2>&1 || { tail -20 $OUT/b_early$v.$r.log; exit 1; }
echo "early=$v run $r: $(tail -1 $OUT/b_early$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/pe -o train -- python3 bench.py --steps 6 --warmup 3 --no-infer > $OUT/prof.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof.log; exit 1; }
f=$(find /tmp/pe -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/train_kernel_trace.csv.gz
python3 scripts/trace_streams.py $OUT/train_kernel_trace.csv.gz > $OUT/train_streams.txt 2>&1 || true
head -16 $OUT/train_streams.txt
