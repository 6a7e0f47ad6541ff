#!/bin/bash
# Round 5 session 27: which aten ops still reach the vendor libraries in fp32 training (innermost repo frames).
set -o pipefail
OUT=gpurun_out/r5s27
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u scripts/torch_prof.py --mode train --fp32 --vendor --out $OUT > $OUT/log.txt 2>&1 || { tail -30 $OUT/log.txt; exit 1; }
cat $OUT/torch_vendor_train.txt
