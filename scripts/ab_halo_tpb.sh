mkdir -p gpurun_out/ab
for t in ${TPBS:-12 16 24 48 12 16 24 48}; do
  RS_HALO_TPB=$t timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/ab/tpb_$t.log 2>&1 || exit 1
  echo "tpb=$t $(tail -1 gpurun_out/ab/tpb_$t.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
