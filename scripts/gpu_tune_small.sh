#!/bin/bash
# Tune RAFT-small's bf16 update-block calls (training 368x496 and the STIR
# tracker's 512x640 inference), then measure config 7 (STIR bf16).
set -o pipefail
mkdir -p gpurun_out/ts
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp raft_stir_amd/conv_tuning.json gpurun_out/ts/conv_tuning.json
timeout -k 10 500 python scripts/tune_conv.py --small --infer-size 512 640 --merge --out gpurun_out/ts/conv_tuning.json > gpurun_out/ts/tune_small_bf16.log 2>&1 || { tail -20 gpurun_out/ts/tune_small_bf16.log; exit 1; }
tail -n 3 gpurun_out/ts/tune_small_bf16.log
cp gpurun_out/ts/conv_tuning.json raft_stir_amd/conv_tuning.json
timeout -k 10 300 python scripts/bench_configs.py --only 7 > gpurun_out/ts/configs.jsonl 2> gpurun_out/ts/configs.err || { tail -20 gpurun_out/ts/configs.err; exit 1; }
cat gpurun_out/ts/configs.jsonl
