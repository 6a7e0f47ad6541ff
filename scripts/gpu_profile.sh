#!/bin/bash
# GPU measurement session: build, short bench (HIP path + stock-PyTorch A/B),
# rocprofv3 kernel stats of the training step and of inference.
# Every GPU step has its own time limit; stop at the first failure.
# Env: BENCH=0 skips the bench, REF_AB=0 skips the stock-PyTorch A/B run,
#      PROF=0 skips profiling.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
test -f raft_stir_amd/_C.so && test -f raft_stir_amd/_host.so || { echo "prebuilt extension missing: run the build on the CPU first"; exit 1; }
if [[ ${BENCH:-1} == 1 ]]; then
timeout -k 10 400 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench_hip.log 2>&1 || { echo BENCH FAILED; tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
fi
if [[ ${REF_AB:-1} == 1 ]]; then
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --reference-ops --no-graph > gpurun_out/bench_ref.log 2>&1 || { echo REF BENCH FAILED; tail -30 gpurun_out/bench_ref.log; exit 1; }
tail -1 gpurun_out/bench_ref.log
fi
if [[ ${PROF:-1} == 1 ]]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof/train -o train -- python3 bench.py --steps 3 --warmup 2 --no-infer > gpurun_out/prof_train.log 2>&1 || { echo PROF TRAIN FAILED; tail -30 gpurun_out/prof_train.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof/infer -o infer -- python3 scripts/infer_only.py --reps 5 > gpurun_out/prof_infer.log 2>&1 || { echo PROF INFER FAILED; tail -30 gpurun_out/prof_infer.log; exit 1; }
find /tmp/prof -name "*stats.csv" -exec cp {} gpurun_out/prof/ \;
ls -la gpurun_out/prof
fi
exit 0
