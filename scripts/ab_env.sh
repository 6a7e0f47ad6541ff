# paired in-situ A/B of schedule switches: each line "<env assignment> pairs/s infer-FPS"
mkdir -p gpurun_out/ab
for e in ${ENVS:-"X=0" "RS_DEFER_ENC=1" "RS_SIDE_PRIO=-1" "X=0" "RS_DEFER_ENC=1" "RS_SIDE_PRIO=-1"}; do
  env $e timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/ab/env.log 2>&1 || exit 1
  echo "$e $(tail -1 gpurun_out/ab/env.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["inference"]["fps"])')"
done
