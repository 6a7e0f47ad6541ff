#!/bin/bash
# Round 5 session 3: conv_v3 MFMA-only / no-loop experiments + PMC counters of tiles 60 / 61 / 77.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/r5s3
mkdir -p $OUT
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen \
  --only gru_zr q_dg --tiles 53 60 61 76 77 78 79 > $OUT/bench_exp.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench_exp.log; exit 1; }
cat $OUT/bench_exp.log
CASES="gru_zr:60:8:46:62 gru_zr:61:8:46:62 gru_zr:77:8:46:62 gru_zr:53:8:46:62" timeout -k 10 600 bash scripts/pmc_update_conv.sh > $OUT/pmc.log 2>&1 || { echo "PMC FAILED"; tail -20 $OUT/pmc.log; exit 1; }
cp gpurun_out/pmc_uc/summary.txt $OUT/pmc_summary.txt
cat $OUT/pmc_summary.txt
