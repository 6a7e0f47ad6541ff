#!/bin/bash
# Round 5 session 13: conv_v3 tiles with pixel-row wave groups (66-68): gate + microbench.
set -o pipefail
OUT=gpurun_out/r5s13
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "v3" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen \
  --only convc2 convf2 conv gru_zr gru_q head zr_dg q_dg head_dg c2_dg cv_dg f2_dg \
  --tiles 61 64 65 66 67 68 > $OUT/bench_train.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench_train.log; exit 1; }
cat $OUT/bench_train.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 1 --hw 55 136 --reps 50 --no-miopen \
  --only convc2 convf2 conv gru_zr gru_q head --tiles 61 65 66 67 68 > $OUT/bench_infer.log 2>&1 || { echo BENCH2 FAILED; tail -20 $OUT/bench_infer.log; exit 1; }
cat $OUT/bench_infer.log
timeout -k 10 300 python -u scripts/bench_enc_v3.py --tiles 61 65 66 67 68 > $OUT/bench_enc.log 2>&1 || { echo BENCH3 FAILED; tail -20 $OUT/bench_enc.log; exit 1; }
cat $OUT/bench_enc.log
