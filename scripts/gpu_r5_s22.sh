#!/bin/bash
# Round 5 session 22: 1x1 GEMM tile 70 -- tests, microbench vs the tuned tiles and hipBLASLt, A/B vs the last commit.
set -o pipefail
OUT=gpurun_out/r5s22
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fused_gpu.py tests/test_enc_conv_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen --gemm \
  --only convc1p mask2 c1_dg m2_dg --tiles 16 17 31 70 > $OUT/bench_train.log 2>&1 || { tail -20 $OUT/bench_train.log; exit 1; }
cat $OUT/bench_train.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 1 --hw 55 136 --reps 50 --no-miopen --gemm \
  --only convc1p mask2 --tiles 16 17 19 70 > $OUT/bench_infer.log 2>&1 || { tail -20 $OUT/bench_infer.log; exit 1; }
cat $OUT/bench_infer.log
run() {  # $1 label, $2 dir, $3 env
  (cd $2 && env $3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
}
for rep in 1 2; do
  run base ab_base X=1 || exit 1
  run new . X=1 || exit 1
done
