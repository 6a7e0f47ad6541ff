#!/bin/bash
# three-stage weight-gradient DMA tiles (variants 6-9), flow_wgrad register
# ring, vectorised tiled OTF backward: gates, microbench, in-situ A/Bs
set -o pipefail
mkdir -p gpurun_out/s21
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_fused_train_gpu.py::test_wgrad_tile_variants" "tests/test_fused_train_gpu.py::test_flow_wgrad" \
  "tests/test_kernels_gpu.py::test_onthefly_tiled_backward" "tests/test_kernels_gpu.py::test_onthefly_corr_fwd_bwd" \
  > gpurun_out/s21/gates.log 2>&1; rc=$?
tail -5 gpurun_out/s21/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 400 python -u scripts/bench_conv.py --hw 46 62 --batch 8 --wgrad 12 --tiles --no-miopen \
  > gpurun_out/s21/wgrad_bench.log 2>&1 || { tail -20 gpurun_out/s21/wgrad_bench.log; exit 1; }
cat gpurun_out/s21/wgrad_bench.log | grep wgrad
for e in "X=1" "RS_WGRAD_NS3=1" "X=1" "RS_WGRAD_NS3=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s21/ab.log 2>&1 || { tail -20 gpurun_out/s21/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s21/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
for args in "--small --alternate-corr" "--alternate-corr"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $args > gpurun_out/s21/otf.log 2>&1 || { tail -20 gpurun_out/s21/otf.log; exit 1; }
  echo "[$args] $(tail -1 gpurun_out/s21/otf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
