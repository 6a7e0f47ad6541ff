#!/bin/bash
# Round 5 session 31: eager step vs the whole step replayed from one hipGraph (--train-graph), same box.
set -o pipefail
OUT=gpurun_out/r5s31
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for rep in 1 2; do
for a in "" "--train-graph"; do
  timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-infer $a > $OUT/ab.log 2>&1 || { tail -30 $OUT/ab.log; exit 1; }
  echo "[${a:-eager}] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pg -o train -- python3 bench.py --steps 8 --warmup 3 --no-infer --train-graph > $OUT/prof_graph.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_graph.log; exit 1; }
f=$(find /tmp/pg -name "*kernel_trace.csv" | head -1); gzip -c $f > $OUT/graph_kernel_trace.csv.gz
python3 scripts/trace_streams.py $OUT/graph_kernel_trace.csv.gz > $OUT/graph_streams.txt 2>&1 || true
head -16 $OUT/graph_streams.txt
