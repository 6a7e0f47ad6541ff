#!/bin/bash
# final check of the end-of-round tree: full GPU suite, smoke, headline bench x2
set -o pipefail
mkdir -p gpurun_out/s30
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s30/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s30/pytest_gpu.log | tail -20
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s30/smoke.log 2>&1 || { tail -20 gpurun_out/s30/smoke.log; exit 1; }
tail -n 1 gpurun_out/s30/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/s30/bench.log 2>&1 && tail -1 gpurun_out/s30/bench.log | tee -a gpurun_out/s30/bench.jsonl | cut -c1-200 || { tail -5 gpurun_out/s30/bench.log; exit 1; }
done
exit $rc
