#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/s17
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/enc_host_profile.py > gpurun_out/s17/enc_host.log 2>&1; head -75 gpurun_out/s17/enc_host.log | cut -c1-160
