#!/bin/bash
# packed-weight refresh after clip_and_step (regression gate), then the
# 3-seed fidelity ensemble again (the s22 one ran with stale packed weights)
set -o pipefail
mkdir -p gpurun_out/s24
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_optim_gpu.py \
  tests/test_graph_train_gpu.py > gpurun_out/s24/gates.log 2>&1; rc=$?
tail -5 gpurun_out/s24/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 1000 python -u scripts/fidelity_ensemble.py --seeds 3 > gpurun_out/s24/fid_ens.log 2>&1; rc=$?
grep -v "amdgpu\|Warning\|sched.step" gpurun_out/s24/fid_ens.log | tail -16
if [[ $rc -ne 0 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/s24/bench.log 2>&1 && tail -1 gpurun_out/s24/bench.log | cut -c1-900
