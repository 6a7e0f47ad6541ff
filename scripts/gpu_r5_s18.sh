#!/bin/bash
# Round 5 session 18: bisect this tree vs the last commit (ab_base/) on one box + kernel stats of both.
set -o pipefail
OUT=gpurun_out/r5s18
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
run() {  # $1 label, $2 dir, $3 env
  (cd $2 && env $3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
}
OFF="RS_AB_CORR_LIB=1 RS_AB_T68=0 RS_AB_SINK_V3=0"
for rep in 1 2; do
  run base ab_base X=1 || exit 1
  run new . X=1 || exit 1
  run new-toggles-off . "$OFF" || exit 1
  run new-toggles-off-nostem . "$OFF RS_AB_STEM=0" || exit 1
done
for d in base new; do
  dir=.; [[ $d == base ]] && dir=ab_base
  (cd $dir && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$d -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer) > $OUT/prof_$d.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$d.log; exit 1; }
  find /tmp/prof_$d -name "*kernel_stats.csv" -exec cp {} $OUT/train_kernel_stats_$d.csv \;
done
ls $OUT
