#!/bin/bash
# full GPU suite after deleting the epilogue-statistics / 128-channel halo
# paths, then the headline bench
set -o pipefail
mkdir -p gpurun_out/s20
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread \
  > gpurun_out/s20/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s20/tests.log | tail -25
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/s20/bench.log 2>&1 && tail -1 gpurun_out/s20/bench.log | cut -c1-900 || { tail -5 gpurun_out/s20/bench.log; exit 1; }
