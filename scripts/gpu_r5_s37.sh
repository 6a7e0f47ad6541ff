#!/bin/bash
# Round 5 session 37: glue-op attribution of the training step; RAFT-small inference and STIR bf16 kernel stats.
set -o pipefail
OUT=gpurun_out/r5s37
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/torch_prof.py --mode train > $OUT/torch_prof.log 2>&1 || { tail -30 $OUT/torch_prof.log; exit 1; }
cp gpurun_out/torch_prof_train.txt $OUT/ 2>/dev/null || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pis -o infer -- python3 scripts/infer_only.py --small --graph --reps 20 > $OUT/prof_infer_small.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_infer_small.log; exit 1; }
find /tmp/pis -name "*kernel_stats.csv" -exec cp {} $OUT/infer_small_kernel_stats.csv \;
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pst -o stir -- python3 scripts/stir_only.py --bf16 --reps 20 > $OUT/prof_stir.log 2>&1 || { echo PROF FAILED; tail -20 $OUT/prof_stir.log; exit 1; }
find /tmp/pst -name "*kernel_stats.csv" -exec cp {} $OUT/stir_bf16_kernel_stats.csv \;
tail -2 $OUT/prof_infer_small.log $OUT/prof_stir.log
