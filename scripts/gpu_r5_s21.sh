#!/bin/bash
# Round 5 session 21: same-box inference kernel stats, last-but-one commit (ab_base/) vs this tree.
set -o pipefail
OUT=gpurun_out/r5s21
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for d in base new; do
  dir=.; [[ $d == base ]] && dir=ab_base
  (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pi_$d -o infer -- python3 scripts/infer_only.py --reps 20) > $OUT/prof_$d.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$d.log; exit 1; }
  find /tmp/pi_$d -name "*kernel_stats.csv" -exec cp {} $OUT/infer_kernel_stats_$d.csv \;
done
for rep in 1 2; do
for d in base new; do
  dir=.; [[ $d == base ]] && dir=ab_base
  (cd $dir && timeout -k 10 300 python bench.py --steps 2 --warmup 1 --infer-reps 100) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$d] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["inference"]["fps"])')"
done
done
