#!/bin/bash
# Round 5 session 35: LDS-staged upflow8 column pass (tests + RAFT-small A/B); OTF backward atomic cost.
set -o pipefail
OUT=gpurun_out/r5s35
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "upflow8" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python scripts/bench_otf_bwd.py > $OUT/otf_bwd.log 2>&1 || { tail -20 $OUT/otf_bwd.log; exit 1; }
cat $OUT/otf_bwd.log
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run base-small ab_base --small || exit 1
  run new-small . --small || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_s -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --small > $OUT/prof_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small.log; exit 1; }
find /tmp/prof_s -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
grep upflow8 $OUT/train_small_kernel_stats.csv
