#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/s5
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_conv.py --batch 8 --hw 46 62 --tiles 16 29 31 45 48 49 50 --only convc2 conv gru_zr gru_q head --reps 20 --no-miopen > gpurun_out/s5/conv_train.log 2>&1 || { tail -20 gpurun_out/s5/conv_train.log; exit 1; }
cat gpurun_out/s5/conv_train.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_fused_train_gpu.py::test_fused_fp32_training_matches_module_graph" \
  "tests/test_model_gpu.py::test_training_grads_match_cpu" tests/test_fused_train_gpu.py::test_fused_training_matches_module_graph \
  > gpurun_out/s5/pytest.log 2>&1; echo "pytest rc=$?"
grep -E "PASS|FAIL|Error|assert|rel" gpurun_out/s5/pytest.log | head -40
timeout -k 10 300 python bench.py --fp32 --steps 10 --warmup 3 --no-infer > gpurun_out/s5/bench_fp32.log 2>&1; tail -3 gpurun_out/s5/bench_fp32.log
