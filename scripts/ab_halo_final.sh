# default tiles-per-block rule vs fixed 12: training pairs/s and graphed inference FPS
mkdir -p gpurun_out/ab
for t in 0 12 0 12; do
  RS_HALO_TPB=$t timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/ab/fin_$t.log 2>&1 || exit 1
  echo "tpb=$t $(tail -1 gpurun_out/ab/fin_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["inference"]["fps"])')"
done
