#!/bin/bash
# wpack gather change gates; whole-step hipGraph vs eager (same box)
set -o pipefail
mkdir -p gpurun_out/s27
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_enc_conv_gpu.py \
  tests/test_enc_geo_gpu.py tests/test_graph_train_gpu.py tests/test_optim_gpu.py > gpurun_out/s27/gates.log 2>&1; rc=$?
tail -3 gpurun_out/s27/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for args in "" "--train-graph" "" "--train-graph"; do
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer $args > gpurun_out/s27/ab.log 2>&1 || { tail -20 gpurun_out/s27/ab.log; exit 1; }
  echo "[$args] $(tail -1 gpurun_out/s27/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
