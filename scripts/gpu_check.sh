#!/bin/bash
# Build + selected GPU tests (TESTS=...) + bench + kernel-stats profile.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
test -f raft_stir_amd/_C.so && test -f raft_stir_amd/_host.so || { echo "prebuilt extension missing: run the build on the CPU first"; exit 1; }
if [[ -n "${TESTS}" ]]; then
  timeout -k 10 900 python -m pytest ${TESTS} -x -q > gpurun_out/pytest.log 2>&1
  rc=$?; tail -15 gpurun_out/pytest.log; [[ $rc -ne 0 ]] && exit $rc
fi
BENCH=${BENCH:-1} REF_AB=${REF_AB:-0} PROF=${PROF:-1} bash scripts/gpu_profile.sh
