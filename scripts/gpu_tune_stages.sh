#!/bin/bash
# Tune the training calls of the reference's later stages (per-GPU batch 6:
# FlyingThings 400x720, Sintel 368x768, KITTI 288x960; scripts/train_*.sh).
set -o pipefail
mkdir -p gpurun_out/tst
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp raft_stir_amd/conv_tuning.json gpurun_out/tst/conv_tuning.json
for sz in "400 720" "368 768" "288 960"; do
  timeout -k 10 400 python scripts/tune_conv.py --batch 6 --size $sz --infer-size 64 64 --merge --out gpurun_out/tst/conv_tuning.json >> gpurun_out/tst/tune.log 2>&1 || { tail -20 gpurun_out/tst/tune.log; exit 1; }
done
grep "sum over" gpurun_out/tst/tune.log
