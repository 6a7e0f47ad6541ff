#!/bin/bash
# three-stage weight-gradient DMA tiles (variants 6-9): correctness vs the
# two-stage twins, microbench at the training shapes, in-situ A/B
set -o pipefail
mkdir -p gpurun_out/s21
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_fused_train_gpu.py::test_wgrad_tile_variants" > gpurun_out/s21/gates.log 2>&1; rc=$?
tail -5 gpurun_out/s21/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u scripts/bench_conv.py --hw 46 62 --batch 8 --wgrad 12 --tiles --no-miopen \
  > gpurun_out/s21/wgrad_bench.log 2>&1 || { tail -20 gpurun_out/s21/wgrad_bench.log; exit 1; }
cat gpurun_out/s21/wgrad_bench.log | grep wgrad
for e in "X=1" "RS_WGRAD_NS3=1" "X=1" "RS_WGRAD_NS3=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s21/ab.log 2>&1 || { tail -20 gpurun_out/s21/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s21/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
