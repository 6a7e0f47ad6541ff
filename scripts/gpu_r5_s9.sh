#!/bin/bash
# Round 5 session 9: encoder 3x3 convs on the weight-streaming tiles: gates + same-box A/B.
set -o pipefail
OUT=gpurun_out/r5s9
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_enc_conv_gpu.py tests/test_model_gpu.py tests/test_fused_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for e in "RS_ENC_V3=0" "X=1" "RS_ENC_V3=0" "X=1"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
