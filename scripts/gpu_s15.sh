#!/bin/bash
# fp32 encoder training on the F32 tiles + one-pass split: tests, fp32 bench + profile
set -o pipefail
mkdir -p gpurun_out/s15
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_enc_f32_train_gpu.py \
  "tests/test_kernels_gpu.py::test_split_bf16_matches_aten" tests/test_model_gpu.py \
  "tests/test_fused_train_gpu.py::test_fused_fp32_training_matches_module_graph" > gpurun_out/s15/tests.log 2>&1; rc=$?
tail -25 gpurun_out/s15/tests.log
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --fp32 --steps 10 --warmup 3 --no-infer > gpurun_out/s15/bench_fp32.log 2>&1 && tail -1 gpurun_out/s15/bench_fp32.log | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf32 -o t -- python3 bench.py --fp32 --steps 3 --warmup 2 --no-infer > gpurun_out/s15/prof32.log 2>&1 || { tail -5 gpurun_out/s15/prof32.log; exit 1; }
find /tmp/pf32 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s15/train_fp32_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s15/train_fp32_kernel_stats.csv 5 2>&1 | head -24 || true
timeout -k 10 300 python scripts/fp32_train_parity.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/s15/parity.log
