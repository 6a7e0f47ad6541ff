#!/bin/bash
# End-of-round session: GPU tests, smoke, headline bench, kernel stats and
# stream timeline, every BASELINE config, RAFT-small bench and the headline
# with the fp32 pyramid (round-2 verdict item 8).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
# a failing test is reported but does not stop the measurements; a crash,
# abort or time limit (124 / 134 / 137 / 139) does
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?
tail -n 3 gpurun_out/final/pytest_gpu.log
if [[ $rc -eq 124 || $rc -eq 134 || $rc -eq 137 || $rc -eq 139 ]]; then echo "pytest rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -n 1 gpurun_out/final/smoke.log
bash scripts/gpu_measure.sh || exit 1
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 --small > gpurun_out/final/bench_small.log 2>&1 || { tail -20 gpurun_out/final/bench_small.log; exit 1; }
tail -n 1 gpurun_out/final/bench_small.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer --corr-dtype float32 > gpurun_out/final/bench_fp32pyr.log 2>&1 || { tail -20 gpurun_out/final/bench_fp32pyr.log; exit 1; }
tail -n 1 gpurun_out/final/bench_fp32pyr.log
PROF=1 bash scripts/gpu_configs.sh || exit 1
