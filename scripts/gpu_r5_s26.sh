#!/bin/bash
# Round 5 session 26: full GPU suite + smoke on the current tree, RAFT-small and headline A/B vs ab_base, small profile.
set -o pipefail
OUT=gpurun_out/r5s26
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --infer-reps 50 $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("inference", {}).get("fps"))')"
}
for rep in 1 2; do
  run base ab_base "" || exit 1
  run new . "" || exit 1
  run base-small ab_base --small || exit 1
  run new-small . --small || exit 1
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_small -o train -- python3 bench.py --steps 6 --warmup 4 --no-infer --small > $OUT/prof_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_small.log; exit 1; }
find /tmp/prof_small -name "*kernel_stats.csv" -exec cp {} $OUT/train_small_kernel_stats.csv \;
