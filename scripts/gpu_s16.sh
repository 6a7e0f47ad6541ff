#!/bin/bash
# regression gates after the fp32 encoder path / optimizer changes + headline bench
set -o pipefail
mkdir -p gpurun_out/s16
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_enc_f32_train_gpu.py \
  tests/test_model_gpu.py tests/test_fused_train_gpu.py tests/test_graph_train_gpu.py tests/test_optim_gpu.py \
  tests/test_enc_conv_gpu.py tests/test_enc_geo_gpu.py > gpurun_out/s16/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s16/tests.log | tail -15
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s16/bench.log 2>&1 && tail -1 gpurun_out/s16/bench.log | cut -c1-600
