#!/bin/bash
# full GPU suite + smoke on the end-of-round tree
set -o pipefail
mkdir -p gpurun_out/s28
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s28/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s28/pytest_gpu.log | tail -20
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s28/smoke.log 2>&1 || { tail -20 gpurun_out/s28/smoke.log; exit 1; }
tail -n 2 gpurun_out/s28/smoke.log
exit $rc
