#!/bin/bash
# One GPU session: build check, GPU tests, smoke, short bench. Each GPU step
# has its own time limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo BUILD FAILED; tail -30 gpurun_out/build.log; exit 1; }
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
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
