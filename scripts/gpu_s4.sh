#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/s4
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/bench_conv.py --batch 8 --hw 46 62 --tiles 16 17 28 29 31 45 47 48 49 50 --only convc2 conv gru_zr gru_q head --reps 20 --no-miopen > gpurun_out/s4/conv_train.log 2>&1 || { tail -20 gpurun_out/s4/conv_train.log; exit 1; }
cat gpurun_out/s4/conv_train.log
timeout -k 10 300 python scripts/bench_conv.py --batch 1 --hw 55 136 --tiles 26 35 36 42 45 48 49 50 --only convc2 conv gru_zr gru_q head --reps 20 --no-miopen > gpurun_out/s4/conv_infer.log 2>&1 || { tail -20 gpurun_out/s4/conv_infer.log; exit 1; }
cat gpurun_out/s4/conv_infer.log
bash scripts/ab_args.sh
