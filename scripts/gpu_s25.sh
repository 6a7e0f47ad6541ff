#!/bin/bash
# new fidelity test (3-seed deterministic fp32 / bf16 ensemble), bench after
# the packed-weight refresh fix
set -o pipefail
mkdir -p gpurun_out/s25
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_train_fidelity_gpu.py \
  > gpurun_out/s25/fid.log 2>&1; rc=$?
grep -E "seed|means|passed|failed|Error" gpurun_out/s25/fid.log | tail -12
if [[ $rc -ne 0 ]]; then exit $rc; fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/s25/bench.log 2>&1 && tail -1 gpurun_out/s25/bench.log | tee -a gpurun_out/s25/bench.jsonl | cut -c1-240 || { tail -5 gpurun_out/s25/bench.log; exit 1; }
done
