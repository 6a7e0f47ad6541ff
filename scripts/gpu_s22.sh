#!/bin/bash
# 3-seed training-fidelity ensemble (fp32 deterministic / bf16 / bf16 deterministic)
set -o pipefail
mkdir -p gpurun_out/s22
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1000 python -u scripts/fidelity_ensemble.py --seeds 3 > gpurun_out/s22/fid_ens.log 2>&1; rc=$?
grep -v "amdgpu\|Warning\|sched.step" gpurun_out/s22/fid_ens.log | tail -14
exit $rc
