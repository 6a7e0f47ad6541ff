set -o pipefail
OUT=gpurun_out/r6s1
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
for it in 1 4 8; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer --iters $it > $OUT/b_it$it.log 2>&1 || { tail -20 $OUT/b_it$it.log; exit 1; }
tail -1 $OUT/b_it$it.log | cut -c1-200
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST FAILED; tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
