# graphed 1088x436 inference FPS (bench.py's inference leg) per RS_HALO_TPB
mkdir -p gpurun_out/ab
for t in ${TPBS:-12 4 2 12 4 2}; do
  RS_HALO_TPB=$t timeout -k 10 200 python bench.py --steps 2 --warmup 1 --infer-reps 50 > gpurun_out/ab/inf_tpb_$t.log 2>&1 || exit 1
  echo "tpb=$t $(tail -1 gpurun_out/ab/inf_tpb_$t.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["inference"]["fps"])')"
done
