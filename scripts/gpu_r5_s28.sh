#!/bin/bash
# Round 5 session 28: fp32 stem training test + fp32 training kernel stats (vendor inventory) + fp32 A/B.
set -o pipefail
OUT=gpurun_out/r5s28
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_stem_gpu.py tests/test_enc_f32_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_f32 -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --fp32 > $OUT/prof_fp32.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_fp32.log; exit 1; }
find /tmp/prof_f32 -name "*kernel_stats.csv" -exec cp {} $OUT/train_fp32_kernel_stats.csv \;
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 10 --warmup 4 --no-infer $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2; do
  run base-fp32 ab_base --fp32 || exit 1
  run new-fp32 . --fp32 || exit 1
done
