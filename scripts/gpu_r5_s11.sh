#!/bin/bash
# Round 5 session 11: wgrad_v3 with per-tap counted LDS waits: gate, microbench, in-situ A/B.
set -o pipefail
OUT=gpurun_out/r5s11
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_train_gpu.py tests/test_determinism_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_conv.py --batch 8 --hw 46 62 --reps 20 --no-miopen --tiles --wgrad 12 --v3wgrad --wvars 0 2 4 \
  --only convc2 convf2 conv gru_zr gru_q head > $OUT/bench_wg.log 2>&1 || { echo BENCH FAILED; tail -20 $OUT/bench_wg.log; exit 1; }
cat $OUT/bench_wg.log
for e in "RS_WGRAD_V3=0" "X=1" "RS_WGRAD_V3=0" "X=1"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
