#!/bin/bash
# Tune the split-bf16 F32 tiles on the fp32 inference calls (RAFT 1088x436 and
# the STIR tracker's RAFT-small 512x640), then measure configs 5 and 6.
set -o pipefail
mkdir -p gpurun_out/f32
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp raft_stir_amd/conv_tuning.json gpurun_out/f32/conv_tuning.json
timeout -k 10 400 python scripts/tune_conv.py --f32 --merge --out gpurun_out/f32/conv_tuning.json > gpurun_out/f32/tune_raft.log 2>&1 || { tail -20 gpurun_out/f32/tune_raft.log; exit 1; }
timeout -k 10 400 python scripts/tune_conv.py --f32 --small --infer-size 512 640 --merge --out gpurun_out/f32/conv_tuning.json > gpurun_out/f32/tune_small.log 2>&1 || { tail -20 gpurun_out/f32/tune_small.log; exit 1; }
tail -2 gpurun_out/f32/tune_raft.log gpurun_out/f32/tune_small.log
cp gpurun_out/f32/conv_tuning.json raft_stir_amd/conv_tuning.json
timeout -k 10 400 python scripts/bench_configs.py --only 5 6 > gpurun_out/f32/configs.jsonl 2> gpurun_out/f32/configs.err || { tail -20 gpurun_out/f32/configs.err; exit 1; }
cat gpurun_out/f32/configs.jsonl
