#!/bin/bash
# split-K fused correlation backward: gates + paired A/B against the hipBLASLt
# path; model / determinism tests; fp32 parity; host op profile
set -o pipefail
mkdir -p gpurun_out/s11
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_corr_volume_backward_fused" "tests/test_kernels_gpu.py::test_allpairs_corr_autograd_bf16" \
  "tests/test_kernels_gpu.py::test_allpairs_corr_autograd_bf16_pyramid" tests/test_determinism_gpu.py > gpurun_out/s11/gates.log 2>&1; rc=$?
tail -8 gpurun_out/s11/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for e in "X=1" "RS_CORR_FUSED_BWD=0" "RS_CORR_BWD_KSPLIT=2" "RS_CORR_BWD_KSPLIT=8" "X=1" "RS_CORR_FUSED_BWD=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s11/ab.log 2>&1 || { tail -20 gpurun_out/s11/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s11/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py > gpurun_out/s11/model.log 2>&1; rc=$?
grep -E "passed|failed|FAIL|Error|assert" gpurun_out/s11/model.log | head -20
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/fp32_train_parity.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/s11/parity.log
timeout -k 10 300 python scripts/host_ops_profile.py > gpurun_out/s11/host_ops.log 2>&1; head -60 gpurun_out/s11/host_ops.log
