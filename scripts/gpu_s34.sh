#!/bin/bash
# final tree (weight-gradient target 1024): full GPU suite, smoke, split-K target A/B
set -o pipefail
mkdir -p gpurun_out/s34
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/s34/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/s34/pytest_gpu.log | tail -20
if [[ $rc -ne 0 && $rc -ne 1 ]]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s34/smoke.log 2>&1 || { tail -20 gpurun_out/s34/smoke.log; exit 1; }
tail -n 1 gpurun_out/s34/smoke.log
for e in "X=1" "RS_WGRAD_BLOCKS=512" "RS_WGRAD_BLOCKS=2048" "X=1" "RS_WGRAD_BLOCKS=512" "RS_WGRAD_BLOCKS=2048"; do
  env $e timeout -k 10 240 python bench.py > gpurun_out/s34/ab.log 2>&1 || { tail -20 gpurun_out/s34/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s34/ab.log | tee -a gpurun_out/s34/bench.jsonl | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
exit $rc
