#!/bin/bash
# cost of the per-step repack after the clip_and_step fix: same-box A/B with
# the stock fused AdamW, and a training kernel profile
set -o pipefail
mkdir -p gpurun_out/s26
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for e in "X=1" "RS_FUSED_ADAMW=0" "X=1" "RS_FUSED_ADAMW=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s26/ab.log 2>&1 || { tail -20 gpurun_out/s26/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s26/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o t -- python3 bench.py --steps 10 --warmup 3 --no-infer > gpurun_out/s26/prof.log 2>&1 || { tail -5 gpurun_out/s26/prof.log; exit 1; }
find /tmp/pt -name "*kernel_stats.csv" -exec cp {} gpurun_out/s26/train_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s26/train_kernel_stats.csv 13 2>&1 | head -40 || true
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr -o t -- python3 bench.py --steps 1 --warmup 3 --no-infer > gpurun_out/s26/trace.log 2>&1 || { tail -5 gpurun_out/s26/trace.log; exit 1; }
find /tmp/tr -name "*kernel_trace.csv" -exec cp {} gpurun_out/s26/train_kernel_trace.csv \;
python scripts/trace_streams.py gpurun_out/s26/train_kernel_trace.csv > gpurun_out/s26/train_streams.txt; head -30 gpurun_out/s26/train_streams.txt; gzip -f gpurun_out/s26/train_kernel_trace.csv
