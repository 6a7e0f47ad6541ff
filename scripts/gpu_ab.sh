#!/bin/bash
# Paired in-situ A/B of environment switches on one box: each line
# "<env> pairs/s infer-FPS".  ENVS: space-separated, commas separate several
# assignments of one arm (e.g. "X=0 RS_ENC_WGRAD=0 X=0").  PRE: an optional
# test command run first (its own limit).
set -o pipefail
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [[ -n "$PRE" ]]; then
  timeout -k 10 400 bash -c "$PRE" > gpurun_out/ab/pre.log 2>&1 || { tail -40 gpurun_out/ab/pre.log; exit 1; }
  tail -3 gpurun_out/ab/pre.log
fi
for e in ${ENVS:-X=0}; do
  env ${e//,/ } timeout -k 10 200 python bench.py --steps 30 --warmup 5 --infer-reps 50 ${BENCH_ARGS} > gpurun_out/ab/env.log 2>&1 || { tail -20 gpurun_out/ab/env.log; exit 1; }
  echo "$e $(tail -1 gpurun_out/ab/env.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["inference"]["fps"])')"
done
