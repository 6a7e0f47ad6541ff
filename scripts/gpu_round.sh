#!/bin/bash
# One GPU session: build check, GPU tests, smoke, short bench. Each GPU step
# has its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
test -f raft_stir_amd/_C.so && test -f raft_stir_amd/_host.so || { echo "prebuilt extension missing: run the build on the CPU first"; exit 1; }
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -40 gpurun_out/pytest_gpu.log; [[ $rc -ne 0 ]] && exit $rc
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -20 gpurun_out/smoke.log; [[ $rc -ne 0 ]] && exit $rc
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup ${BENCH_WARMUP:-3} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
  rc=$?; tail -20 gpurun_out/bench.log; [[ $rc -ne 0 ]] && exit $rc
fi
exit 0
