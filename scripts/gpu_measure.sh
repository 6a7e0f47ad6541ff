#!/bin/bash
# One measurement session: GPU tests (optional), the bench line, a one-step
# kernel trace of training (per-queue breakdown) and rocprofv3 kernel stats
# of training and of graphed inference.  Every GPU step has its own limit;
# the chain stops at the first failure.
#   TESTS=1 runs pytest -m gpu first; BENCH_ARGS / INFER_ARGS pass through.
set -o pipefail
mkdir -p gpurun_out/m
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
test -f raft_stir_amd/_C.so || { echo "prebuilt extension missing"; exit 1; }
if [[ ${TESTS:-0} == 1 ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/m/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/m/pytest_gpu.log; [[ $rc -ne 0 ]] && exit $rc
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 ${BENCH_ARGS} > gpurun_out/m/bench.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/m/bench.log; exit 1; }
tail -1 gpurun_out/m/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr -o t -- python3 bench.py --steps 1 --warmup 3 --no-infer ${BENCH_ARGS} > gpurun_out/m/trace.log 2>&1 || { echo TRACE FAILED; tail -30 gpurun_out/m/trace.log; exit 1; }
find /tmp/tr -name "*kernel_trace.csv" -exec cp {} gpurun_out/m/train_kernel_trace.csv \;
python scripts/trace_streams.py gpurun_out/m/train_kernel_trace.csv > gpurun_out/m/train_streams.txt && gzip -f gpurun_out/m/train_kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt -o train -- python3 bench.py --steps 3 --warmup 2 --no-infer ${BENCH_ARGS} > gpurun_out/m/prof_train.log 2>&1 || { echo PROF TRAIN FAILED; tail -30 gpurun_out/m/prof_train.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pi -o infer -- python3 scripts/infer_only.py --graph --reps 5 ${INFER_ARGS} > gpurun_out/m/prof_infer.log 2>&1 || { echo PROF INFER FAILED; tail -30 gpurun_out/m/prof_infer.log; exit 1; }
find /tmp/pt /tmp/pi -name "*kernel_stats.csv" -exec cp {} gpurun_out/m/ \;
ls gpurun_out/m
exit 0
