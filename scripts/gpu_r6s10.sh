set -o pipefail
OUT=gpurun_out/r6s10
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for e in X=0 RS_HALO_MIN_P=300000 X=0 RS_HALO_MIN_P=300000; do
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  echo "$e $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done | tee $OUT/ab.txt
timeout -k 10 600 python scripts/bench_dataloader.py --ranks 8 --workers 1 --batches 40 --files 2048 > $OUT/feed8x1.log 2>&1 || { tail -20 $OUT/feed8x1.log; exit 1; }
tail -1 $OUT/feed8x1.log
for e in RS_NORM_REDUCE_BLOCKS=512 RS_NORM_REDUCE_BLOCKS=1024 RS_NORM_REDUCE_BLOCKS=2048 RS_NORM_REDUCE_BLOCKS=512 RS_NORM_REDUCE_BLOCKS=1024 RS_NORM_REDUCE_BLOCKS=2048; do
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  echo "$e $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done | tee $OUT/ab_norm.txt
