#!/bin/bash
# Same-box A/B of the working tree against a baseline worktree (box-to-box
# spread on the pool is 3-5 %, so changes are judged by paired runs on one box).
#
#   git worktree add ab_base <commit>; (cd ab_base && python -c "from raft_stir_amd.build import build_all; build_all()")
#   gpurun -- 'PRE="python -m pytest tests/test_x_gpu.py -q" REPS=3 BENCH_ARGS="--no-infer" bash scripts/gpu_ab_tree.sh'
#
# PRE: optional test command run first (its own limit); REPS: interleaved
# base / new pairs; BENCH_ARGS: extra bench.py flags (--small, --alternate-corr,
# --no-infer, ...).  One line per run: "[arm] pairs/s ms/step infer-FPS".
set -o pipefail
OUT=gpurun_out/ab_tree
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
BASE=${BASE:-ab_base}
if [[ -n "$PRE" ]]; then
  timeout -k 10 600 bash -c "$PRE" > $OUT/pre.log 2>&1 || { tail -40 $OUT/pre.log; exit 1; }
  tail -2 $OUT/pre.log
fi
for rep in $(seq ${REPS:-2}); do
  for arm in base new; do
    if [ $arm = base ]; then D=$BASE; else D=.; fi
    (cd $D && timeout -k 10 400 python bench.py --steps 30 --warmup 5 --infer-reps 50 ${BENCH_ARGS}) > $OUT/$arm.log 2>&1 \
      || { tail -30 $OUT/$arm.log; exit 1; }
    echo "[$arm] $(tail -1 $OUT/$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("inference") or {}).get("fps"))')" | tee -a $OUT/ab.txt
  done
done
