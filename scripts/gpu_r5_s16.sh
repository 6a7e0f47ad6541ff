#!/bin/bash
# Round 5 session 16: stem weight gradient rewrite + row-per-block fold: tests + microbench.
set -o pipefail
OUT=gpurun_out/r5s16
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_stem_gpu.py tests/test_kernels_gpu.py -k "stem or corr_volume_backward or pyr_grad_fold" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/bench_stem.py > $OUT/bench_stem.log 2>&1 || { tail -20 $OUT/bench_stem.log; exit 1; }
cat $OUT/bench_stem.log
timeout -k 10 300 python -u scripts/bench_corr_bwd.py > $OUT/bench_corr_bwd.log 2>&1 || { tail -20 $OUT/bench_corr_bwd.log; exit 1; }
cat $OUT/bench_corr_bwd.log
