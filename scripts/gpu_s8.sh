#!/bin/bash
# fp32 parity vs the CPU oracle, fused corr backward + deterministic OTF tests,
# paired A/B of the fused corr backward, host-side op profile, fp32 profile
set -o pipefail
mkdir -p gpurun_out/s8
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread "tests/test_kernels_gpu.py::test_onthefly_tiled_forward" "tests/test_kernels_gpu.py::test_onthefly_corr_fwd_bwd" "tests/test_kernels_gpu.py::test_onthefly_matches_allpairs" > gpurun_out/s8/otf.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/s8/otf.log | head -30
if [[ $rc -ne 0 && $rc -ne 1 ]]; then tail -20 gpurun_out/s8/otf.log; exit $rc; fi
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_corr_volume_backward_fused" "tests/test_kernels_gpu.py::test_allpairs_corr_autograd_bf16" \
  "tests/test_kernels_gpu.py::test_allpairs_corr_autograd_bf16_pyramid" tests/test_determinism_gpu.py "tests/test_kernels_gpu.py::test_corr_volume_pyramid" tests/test_model_gpu.py > gpurun_out/s8/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" gpurun_out/s8/pytest.log | head -30
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python scripts/fp32_train_parity.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/s8/parity.log
timeout -k 10 300 python scripts/fp32_train_parity.py --small 2>&1 | grep -v amdgpu.ids | tee gpurun_out/s8/parity_small.log
for rep in 1 2; do for e in "X=1" "RS_CORR_FUSED_BWD=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s8/ab.log 2>&1 || { tail -20 gpurun_out/s8/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s8/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done; done
timeout -k 10 300 python scripts/host_ops_profile.py > gpurun_out/s8/host_ops.log 2>&1; head -70 gpurun_out/s8/host_ops.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof32 -o t -- python3 bench.py --fp32 --steps 3 --warmup 2 --no-infer > gpurun_out/s8/prof32.log 2>&1 || { tail -5 gpurun_out/s8/prof32.log; exit 1; }
find /tmp/prof32 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s8/train_fp32_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s8/train_fp32_kernel_stats.csv 3 2>&1 | head -30 || true
