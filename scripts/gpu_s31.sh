#!/bin/bash
# double-buffered all-pairs volume kernel: gates, microbench and inference /
# training A/B against the one-stage kernel (default; RS_CORR_FLAT_DB=1 is the two-stage one), same box
set -o pipefail
mkdir -p gpurun_out/s31
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  > gpurun_out/s31/gates.log 2>&1; rc=$?
tail -3 gpurun_out/s31/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
RS_CORR_FLAT_DB=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_model_gpu.py > gpurun_out/s31/gates_db.log 2>&1; rc=$?
tail -3 gpurun_out/s31/gates_db.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for e in "X=1" "RS_CORR_FLAT_DB=1" "X=1" "RS_CORR_FLAT_DB=1"; do
  env $e timeout -k 10 120 python scripts/bench_corr.py --hw 46 62 --batch 8 --reps 20 2>&1 | grep -v amdgpu | sed "s/^/[$e] /" | head -2
  env $e timeout -k 10 120 python scripts/bench_corr.py --hw 55 136 --batch 1 --reps 20 2>&1 | grep -v amdgpu | sed "s/^/[$e] /" | sed -n 2p
done
for e in "X=1" "RS_CORR_FLAT_DB=1" "X=1" "RS_CORR_FLAT_DB=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --infer-reps 100 > gpurun_out/s31/ab.log 2>&1 || { tail -20 gpurun_out/s31/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s31/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
