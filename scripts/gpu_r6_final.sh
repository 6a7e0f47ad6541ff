set -o pipefail
OUT=gpurun_out/r6final
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
tail -1 $OUT/bench_default.log
for a in "--steps 30 --warmup 5" "--small --steps 40 --warmup 5"; do
  timeout -k 10 400 python bench.py $a > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  tail -1 $OUT/b.log >> $OUT/bench.jsonl
done
cat $OUT/bench.jsonl | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); c=d['config']; i=d.get('inference') or {}
    print(c['model'][:12], c.get('train_step'), d['value'], d['ms_per_step'], i.get('fps'), i.get('ms_per_pair'))
"
# per-kernel time of the training step and of the inference forward (no counters)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_train -o k -- python bench.py --steps 10 --warmup 3 --no-infer > $OUT/prof_train.log 2>&1 || { tail -20 $OUT/prof_train.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_infer -o k -- python bench.py --steps 1 --warmup 1 --infer-reps 25 > $OUT/prof_infer.log 2>&1 || { tail -20 $OUT/prof_infer.log; exit 1; }
find $OUT -name '*kernel_stats.csv' | head -5
