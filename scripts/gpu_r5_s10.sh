#!/bin/bash
# Round 5 session 10: encoder v3 A/B (session 9) + the all-taps weight gradient (wgrad_v3) gate and microbench.
set -o pipefail
OUT=gpurun_out/r5s10
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py -k "wgrad_v3" > $OUT/pytest_wg3.log 2>&1 || { echo PYTEST WG3 FAILED; tail -30 $OUT/pytest_wg3.log; exit 1; }
tail -2 $OUT/pytest_wg3.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen --tiles --wgrad 12 --v3wgrad --wvars 0 1 2 4 \
  --only convc2 convf2 conv gru_zr gru_q head > $OUT/bench_wg.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench_wg.log; exit 1; }
cat $OUT/bench_wg.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_enc_conv_gpu.py tests/test_model_gpu.py tests/test_fused_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for e in "RS_ENC_V3=0" "X=1" "RS_ENC_V3=0" "X=1"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
