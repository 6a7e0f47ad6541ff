#!/bin/bash
# fp32 training bench + profile, the full bench-config table, fidelity probe
set -o pipefail
mkdir -p gpurun_out/s14
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python bench.py --fp32 --steps 10 --warmup 3 > gpurun_out/s14/bench_fp32.log 2>&1 && tail -1 gpurun_out/s14/bench_fp32.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pf32 -o t -- python3 bench.py --fp32 --steps 3 --warmup 2 --no-infer > gpurun_out/s14/prof32.log 2>&1 || { tail -5 gpurun_out/s14/prof32.log; exit 1; }
find /tmp/pf32 -name "*kernel_stats.csv" -exec cp {} gpurun_out/s14/train_fp32_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s14/train_fp32_kernel_stats.csv 5 2>&1 | head -30 || true
timeout -k 10 600 python scripts/bench_configs.py > gpurun_out/s14/configs.log 2>&1; tail -8 gpurun_out/s14/configs.log | cut -c1-400
timeout -k 10 500 python -u scripts/fidelity_probe.py > gpurun_out/s14/fidelity.log 2>&1; cat gpurun_out/s14/fidelity.log | grep -v amdgpu
