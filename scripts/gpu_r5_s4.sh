#!/bin/bash
# Round 5 session 4: batched 32x32 epilogue (conv_v2 / conv_v3): correctness + microbench.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5s4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py tests/test_fused_train_gpu.py \
  > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen \
  --only convc2 convf2 conv gru_zr gru_q head zr_dg q_dg head_dg c2_dg cv_dg f2_dg \
  --tiles 52 53 54 60 61 62 63 64 > $OUT/bench_train.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench_train.log; exit 1; }
cat $OUT/bench_train.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 1 --hw 55 136 --reps 50 --no-miopen \
  --only convc2 convf2 conv gru_zr gru_q head \
  --tiles 45 46 35 36 26 60 61 62 63 64 > $OUT/bench_infer.log 2>&1 || { echo "BENCH2 FAILED"; tail -20 $OUT/bench_infer.log; exit 1; }
cat $OUT/bench_infer.log
