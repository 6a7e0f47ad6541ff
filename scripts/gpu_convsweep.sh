#!/bin/bash
# Conv tile sweep (training + inference shapes) incl. halo tiles and the
# hipBLASLt plain-GEMM lower bound; then kernel-stat profiles.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
test -f raft_stir_amd/_C.so || { echo "prebuilt extension missing"; exit 1; }
TILES=${TILES:-"16 17 20 24 25 26 29 31 33"}
timeout -k 10 300 python -u scripts/bench_conv.py --hw 46 62 --batch 8 --reps 30 --tiles $TILES --gemm --no-miopen > gpurun_out/conv_train.log 2>&1 || { tail -20 gpurun_out/conv_train.log; exit 1; }
cat gpurun_out/conv_train.log
timeout -k 10 300 python -u scripts/bench_conv.py --hw 55 136 --batch 1 --reps 50 --tiles $TILES --gemm --no-miopen > gpurun_out/conv_infer.log 2>&1 || { tail -20 gpurun_out/conv_infer.log; exit 1; }
cat gpurun_out/conv_infer.log
