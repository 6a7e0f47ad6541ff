#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/s6
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/fp32_train_parity.py > gpurun_out/s6/parity.log 2>&1; cat gpurun_out/s6/parity.log | grep -v amdgpu.ids
timeout -k 10 300 python scripts/fp32_train_parity.py --small > gpurun_out/s6/parity_small.log 2>&1; cat gpurun_out/s6/parity_small.log | grep -v amdgpu.ids
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof32 -o t -- python3 bench.py --fp32 --steps 3 --warmup 2 --no-infer > gpurun_out/s6/prof.log 2>&1 || { tail -5 gpurun_out/s6/prof.log; exit 1; }
find /tmp/prof32 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s6/train_fp32_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s6/train_fp32_kernel_stats.csv 2>&1 | head -40 || true
