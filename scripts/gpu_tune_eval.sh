#!/bin/bash
# Tune the update-block calls of the evaluation shapes (KITTI 1242x375 and
# Sintel's 1024x436) for bf16 and fp32, then measure config 4 (KITTI).
set -o pipefail
mkdir -p gpurun_out/te
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp raft_stir_amd/conv_tuning.json gpurun_out/te/conv_tuning.json
for sz in "375 1242" "436 1024"; do
  for m in "" "--f32"; do
    timeout -k 10 400 python scripts/tune_conv.py --infer-only $m --infer-size $sz --merge --out gpurun_out/te/conv_tuning.json >> gpurun_out/te/tune.log 2>&1 || { tail -20 gpurun_out/te/tune.log; exit 1; }
  done
done
grep "sum over" gpurun_out/te/tune.log
cp gpurun_out/te/conv_tuning.json raft_stir_amd/conv_tuning.json
timeout -k 10 300 python scripts/bench_configs.py --only 4 > gpurun_out/te/configs.jsonl 2> gpurun_out/te/configs.err || { tail -20 gpurun_out/te/configs.err; exit 1; }
cat gpurun_out/te/configs.jsonl
