#!/bin/bash
# Round 5 session 19: full GPU suite + smoke, A/B vs the last-but-one commit (ab_base/), vendor-kernel inventory
# of the fp32 and RAFT-small training steps.
set -o pipefail
OUT=gpurun_out/r5s19
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
run() {  # $1 label, $2 dir, $3 env
  (cd $2 && env $3 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
}
for rep in 1 2; do
  run base ab_base X=1 || exit 1
  run new . X=1 || exit 1
done
for m in fp32 small; do
  args="--fp32"; [[ $m == small ]] && args="--small"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$m -o train -- python3 bench.py --steps 4 --warmup 2 --no-infer $args > $OUT/prof_$m.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_$m.log; exit 1; }
  find /tmp/prof_$m -name "*kernel_stats.csv" -exec cp {} $OUT/train_${m}_kernel_stats.csv \;
  tail -1 $OUT/prof_$m.log
done
ls $OUT
