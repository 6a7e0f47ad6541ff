set -o pipefail
OUT=gpurun_out/r6s23
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 30 > $OUT/b.$r.log 2>&1 || { tail -20 $OUT/b.$r.log; exit 1; }
tail -1 $OUT/b.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("headline", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
done
timeout -k 10 300 python bench.py --small --steps 30 --warmup 5 --infer-reps 30 > $OUT/bs.log 2>&1 || { tail -20 $OUT/bs.log; exit 1; }
tail -1 $OUT/bs.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("small", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_t -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_train.log; exit 1; }
find /tmp/pe_t -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats.csv \;
