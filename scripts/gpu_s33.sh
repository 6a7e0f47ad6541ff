#!/bin/bash
# knob sweep on the final tree, same box: norm reduction grid, weight-gradient
# split-K target, conv XCD remap
set -o pipefail
mkdir -p gpurun_out/s33
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for e in "X=1" "RS_NORM_RED_BLOCKS=256" "RS_NORM_RED_BLOCKS=1024" "RS_WGRAD_BLOCKS=1024" "RS_WGRAD_BLOCKS=4096" "RS_CONV_XCD_REMAP=0" \
         "X=1" "RS_NORM_RED_BLOCKS=256" "RS_NORM_RED_BLOCKS=1024" "RS_WGRAD_BLOCKS=1024" "RS_WGRAD_BLOCKS=4096" "RS_CONV_XCD_REMAP=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/s33/ab.log 2>&1 || { tail -20 gpurun_out/s33/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s33/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
