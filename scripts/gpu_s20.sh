#!/bin/bash
# regression gates after deleting the epilogue-statistics / 128-channel halo
# paths, headline bench, 3-seed fidelity ensemble
set -o pipefail
mkdir -p gpurun_out/s20
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_norm_fused_gpu.py \
  tests/test_enc_conv_gpu.py tests/test_enc_geo_gpu.py tests/test_stem_gpu.py tests/test_conv_f32_gpu.py \
  tests/test_norm_gpu.py tests/test_model_gpu.py tests/test_fused_train_gpu.py tests/test_determinism_gpu.py \
  > gpurun_out/s20/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s20/tests.log | tail -15
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s20/bench.log 2>&1 && tail -1 gpurun_out/s20/bench.log | cut -c1-700 || exit 1
timeout -k 10 900 python -u scripts/fidelity_ensemble.py --seeds 3 > gpurun_out/s20/fid_ens.log 2>&1; grep -v "amdgpu\|Warning\|sched.step" gpurun_out/s20/fid_ens.log | tail -14
