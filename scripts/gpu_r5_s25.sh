#!/bin/bash
# Round 5 session 25: register-blocked narrow wgrad -- tests, RAFT-small A/B, kernel stats.
set -o pipefail
OUT=gpurun_out/r5s25
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_sconv_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for rep in 1 2; do
  run base-small ab_base --small || exit 1
  run new-small . --small || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_small -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --small > $OUT/prof_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small.log; exit 1; }
find /tmp/prof_small -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
(cd ab_base && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_small_b -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --small) > $OUT/prof_small_base.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small_base.log; exit 1; }
find /tmp/prof_small_b -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats_base.csv \;
