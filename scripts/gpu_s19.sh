#!/bin/bash
# stream priorities: encoder backward vs the deferred weight gradients
set -o pipefail
mkdir -p gpurun_out/s19
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for e in "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1" "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s19/ab.log 2>&1 || { tail -20 gpurun_out/s19/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s19/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
