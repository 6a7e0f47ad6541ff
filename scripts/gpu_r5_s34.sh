#!/bin/bash
# Round 5 session 34: two-pass upflow8 backward (tests + RAFT-small A/B), every BASELINE config, RAFT-small
# inference, RAFT-small on-the-fly-correlation training profile.
set -o pipefail
OUT=gpurun_out/r5s34
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "upflow8" tests/test_sconv_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run base-small ab_base --small || exit 1
  run new-small . --small || exit 1
done
timeout -k 10 600 python scripts/bench_configs.py --out $OUT/bench_configs.jsonl > $OUT/bench_configs.log 2>&1 || { tail -30 $OUT/bench_configs.log; exit 1; }
cat $OUT/bench_configs.jsonl
timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/infer_small.log 2>&1 || { tail -20 $OUT/infer_small.log; exit 1; }
tail -3 $OUT/infer_small.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_so -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --small --alternate-corr > $OUT/prof_small_otf.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small_otf.log; exit 1; }
find /tmp/prof_so -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_otf_kernel_stats.csv \;
tail -1 $OUT/prof_small_otf.log
