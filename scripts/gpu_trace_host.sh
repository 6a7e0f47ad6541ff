#!/bin/bash
# Host/device timeline of the training step: rocprofv3 kernel + HIP runtime
# API traces of bench.py, joined by scripts/trace_host.py.
set -o pipefail
mkdir -p gpurun_out/trace_host
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d /tmp/trh -o t -- \
  python3 bench.py --steps 3 --warmup 3 --no-infer ${BENCH_ARGS} > gpurun_out/trace_host/log 2>&1 || { tail -20 gpurun_out/trace_host/log; exit 1; }
python3 scripts/trace_host.py /tmp/trh > gpurun_out/trace_host/report.txt 2>&1; cat gpurun_out/trace_host/report.txt
find /tmp/trh -name "*kernel_trace.csv" -exec gzip -c {} \; > gpurun_out/trace_host/kt.csv.gz
python3 scripts/trace_streams.py gpurun_out/trace_host/kt.csv.gz > gpurun_out/trace_host/streams.txt 2>&1 || true
