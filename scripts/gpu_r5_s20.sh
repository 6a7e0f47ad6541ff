#!/bin/bash
# Round 5 session 20: norm / corr / stem tests + A/B vs the last-but-one commit (ab_base/) + kernel stats.
set -o pipefail
OUT=gpurun_out/r5s20
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_norm_gpu.py tests/test_norm_fused_gpu.py tests/test_stem_gpu.py tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # $1 label, $2 dir, $3 env
  (cd $2 && env $3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
}
for rep in 1 2; do
  run base ab_base X=1 || exit 1
  run new . X=1 || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_new -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer > $OUT/prof_new.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_new.log; exit 1; }
find /tmp/prof_new -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats_new.csv \;
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_f32 -o train -- python3 bench.py --steps 8 --warmup 4 --no-infer --fp32 > $OUT/prof_fp32.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_fp32.log; exit 1; }
find /tmp/prof_f32 -name "*kernel_stats.csv" -exec cp {} $OUT/train_fp32_kernel_stats.csv \;
tail -1 $OUT/prof_fp32.log
