#!/bin/bash
# paired in-situ A/B of bench.py argument sets on one box, interleaved:
#   ARGS=("" "--train-graph") bash scripts/ab_args.sh   (ARGSTR: '|'-separated alternative)
set -o pipefail
mkdir -p gpurun_out/ab
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
IFS='|' read -ra SETS <<< "${ARGSTR:-|--train-graph}"
for rep in 1 2; do
  for s in "${SETS[@]}"; do
    timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer $s > gpurun_out/ab/args.log 2>&1 || { tail -20 gpurun_out/ab/args.log; exit 1; }
    echo "[$s] $(tail -1 gpurun_out/ab/args.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
  done
done
