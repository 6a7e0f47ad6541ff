#!/bin/bash
# Round 5 session 17: stem wgrad + row fold tests/bench, then same-box A/B of this tree vs the last commit (ab_base/).
set -o pipefail
OUT=gpurun_out/r5s17
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_stem_gpu.py tests/test_kernels_gpu.py -k "stem or corr_volume_backward or pyr_grad_fold" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python -u scripts/bench_stem.py > $OUT/bench_stem.log 2>&1 || { tail -20 $OUT/bench_stem.log; exit 1; }
cat $OUT/bench_stem.log
timeout -k 10 300 python -u scripts/bench_corr_bwd.py > $OUT/bench_corr_bwd.log 2>&1 || { tail -20 $OUT/bench_corr_bwd.log; exit 1; }
cat $OUT/bench_corr_bwd.log
run() {  # $1 label, $2 dir, $3 env
  (cd $2 && env $3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
}
for rep in 1 2; do
  run base ab_base X=1 || exit 1
  run new . X=1 || exit 1
  run new-nostem . RS_AB_STEM=0 || exit 1
done
