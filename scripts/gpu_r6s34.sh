set -o pipefail
OUT=gpurun_out/r6s34
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sconv_gpu.py tests/test_sconv_train_gpu.py tests/test_model_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -1 $OUT/test.log
for r in 1 2; do
timeout -k 10 300 python bench.py --small --steps 40 --warmup 5 --infer-reps 40 > $OUT/b_small.$r.log 2>&1 || { tail -20 $OUT/b_small.$r.log; exit 1; }
tail -1 $OUT/b_small.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("small", d["value"], d["ms_per_step"], d["config"]["train_step"], d["inference"]["ms_per_pair"])'
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps -o trains -- python3 bench.py --small --eager --steps 8 --warmup 3 --no-infer > $OUT/prof_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small.log; exit 1; }
find /tmp/ps -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
grep "sconv" $OUT/train_small_kernel_stats.csv | cut -c1-120
