#!/bin/bash
# kernel-only trace of the training step (low overhead) -> per-queue timeline
set -o pipefail
mkdir -p gpurun_out/s12
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/trk -o t -- \
  python3 bench.py --steps 3 --warmup 3 --no-infer > gpurun_out/s12/log 2>&1 || { tail -20 gpurun_out/s12/log; exit 1; }
find /tmp/trk -name "*kernel_trace.csv" -exec gzip -c {} \; > gpurun_out/s12/kt.csv.gz
python3 scripts/trace_streams.py gpurun_out/s12/kt.csv.gz > gpurun_out/s12/streams.txt 2>&1; head -110 gpurun_out/s12/streams.txt
