#!/bin/bash
# end-of-round measurements: headline bench, training stream trace, training /
# inference kernel stats (scripts/gpu_measure.sh), RAFT-small, fp32 training,
# on-the-fly training, every BASELINE config with STIR / fp32 kernel stats
set -o pipefail
mkdir -p gpurun_out/s23
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
bash scripts/gpu_measure.sh || exit 1
for args in "--small" "--fp32 --no-infer" "--alternate-corr --no-infer" "--small --alternate-corr --no-infer"; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --infer-reps 50 $args > gpurun_out/s23/b.log 2>&1 || { tail -20 gpurun_out/s23/b.log; exit 1; }
  echo "[$args]"; tail -1 gpurun_out/s23/b.log | tee -a gpurun_out/s23/bench_lines.jsonl | cut -c1-300
done
PROF=1 bash scripts/gpu_configs.sh || exit 1
