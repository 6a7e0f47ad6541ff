#!/bin/bash
# Round 5 session 8: weight-streaming tiles on the encoders' stride-1 3x3 convs (microbench) + tile 65 gate.
set -o pipefail
OUT=gpurun_out/r5s8
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k v3 > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_enc_v3.py --tiles 60 61 63 65 > $OUT/bench_enc.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench_enc.log; exit 1; }
cat $OUT/bench_enc.log
