#!/bin/bash
# Round 5 session 2: conv_v3 timing experiments on the 1x5 convs (tiles 70-76, RS_V3_EXP build).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5s2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k v3 > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen \
  --only gru_zr gru_q zr_dg q_dg --tiles 53 60 61 70 71 72 73 74 75 76 > $OUT/bench_exp.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench_exp.log; exit 1; }
cat $OUT/bench_exp.log
