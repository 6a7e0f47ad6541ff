#!/bin/bash
# Every BASELINE config (scripts/bench_configs.py) plus rocprofv3 kernel
# stats of the STIR point tracker (bf16 and fp32) and of fp32 RAFT inference.
set -o pipefail
mkdir -p gpurun_out/cfg
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python scripts/bench_configs.py --only ${ONLY:-2 4 5 6 7} > gpurun_out/cfg/configs.jsonl 2> gpurun_out/cfg/configs.err || { tail -30 gpurun_out/cfg/configs.err; exit 1; }
cat gpurun_out/cfg/configs.jsonl
if [[ ${PROF:-1} == 1 ]]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sb -o stir_bf16 -- python3 scripts/stir_only.py --bf16 --reps 20 > gpurun_out/cfg/stir_bf16.log 2>&1 || { tail -20 gpurun_out/cfg/stir_bf16.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sf -o stir_fp32 -- python3 scripts/stir_only.py --reps 20 > gpurun_out/cfg/stir_fp32.log 2>&1 || { tail -20 gpurun_out/cfg/stir_fp32.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rf -o infer_fp32 -- python3 scripts/infer_only.py --graph --fp32 --reps 20 > gpurun_out/cfg/infer_fp32.log 2>&1 || { tail -20 gpurun_out/cfg/infer_fp32.log; exit 1; }
find /tmp/sb /tmp/sf /tmp/rf -name "*kernel_stats.csv" -exec cp {} gpurun_out/cfg/ \;
tail -1 gpurun_out/cfg/stir_bf16.log gpurun_out/cfg/stir_fp32.log gpurun_out/cfg/infer_fp32.log
fi
exit 0
