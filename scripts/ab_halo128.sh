# layer3 (128-ch) encoder convs on the halo kernel (RS_ENC_HALO128=1) or the implicit-GEMM tiles (0)
mkdir -p gpurun_out/ab
for t in 1 0 1 0; do
  RS_ENC_HALO128=$t timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/ab/h128_$t.log 2>&1 || exit 1
  echo "halo128=$t $(tail -1 gpurun_out/ab/h128_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["inference"]["fps"])')"
done
