#!/bin/bash
# conv_v2 tile 54 (192 Cout x 4x32 px): gate, retune with it, A/B against the shipped table
set -o pipefail
mkdir -p gpurun_out/s29
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_fused_gpu.py::test_conv_v2_tiles_vs_conv2d" > gpurun_out/s29/gates.log 2>&1; rc=$?
tail -3 gpurun_out/s29/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
cp raft_stir_amd/conv_tuning.json gpurun_out/s29/conv_tuning_before.json
timeout -k 10 600 python -u scripts/tune_conv.py --merge > gpurun_out/s29/tune.log 2>&1 || { tail -20 gpurun_out/s29/tune.log; exit 1; }
grep -E "best t54|sum over" gpurun_out/s29/tune.log | head -30
cp raft_stir_amd/conv_tuning.json gpurun_out/s29/conv_tuning.json
for e in "RS_CONV_TUNING_FILE=gpurun_out/s29/conv_tuning_before.json" "X=1" "RS_CONV_TUNING_FILE=gpurun_out/s29/conv_tuning_before.json" "X=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/s29/ab.log 2>&1 || { tail -20 gpurun_out/s29/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s29/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
