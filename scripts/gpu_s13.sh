#!/bin/bash
# split update-block weight gradients: fused-training gradient tests + paired A/B
set -o pipefail
mkdir -p gpurun_out/s13
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_train_gpu.py \
  tests/test_ddp_gpu.py > gpurun_out/s13/tests.log 2>&1; rc=$?
tail -6 gpurun_out/s13/tests.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for e in "X=1" "RS_WGRAD_SPLIT=0" "X=1" "RS_WGRAD_SPLIT=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s13/ab.log 2>&1 || { tail -20 gpurun_out/s13/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s13/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
