#!/bin/bash
# Round 5 session 39: training metrics inside the loss kernel, convex backward into the padded d_mask (tests + A/B).
set -o pipefail
OUT=gpurun_out/r5s39
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_loss_gpu.py tests/test_kernels_gpu.py tests/test_fused_train_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for rep in 1 2 3; do
for arm in base new; do
  if [ $arm = base ]; then D=ab_base; else D=.; fi
  (cd $D && timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-infer) > $OUT/ab_$arm.log 2>&1 || { tail -30 $OUT/ab_$arm.log; exit 1; }
  echo "[$arm] $(tail -1 $OUT/ab_$arm.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("final_loss"))')" | tee -a $OUT/ab.txt
done
done
