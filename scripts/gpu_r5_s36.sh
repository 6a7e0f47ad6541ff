#!/bin/bash
# Round 5 session 36: OTF tiled backward on MFMA (tests, microbench, RAFT-small / RAFT OTF training A/B).
set -o pipefail
OUT=gpurun_out/r5s36
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "onthefly" tests/test_determinism_gpu.py tests/test_fused_train_gpu.py -k "onthefly or otf or determin" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python scripts/bench_otf_bwd.py > $OUT/otf_bwd.log 2>&1 || { tail -20 $OUT/otf_bwd.log; exit 1; }
cat $OUT/otf_bwd.log
run() {  # $1 label, $2 dir, $3 args
  (cd $2 && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $3) > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$1] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/ab.txt
}
for rep in 1 2; do
  run base-small-otf ab_base "--small --alternate-corr" || exit 1
  run new-small-otf . "--small --alternate-corr" || exit 1
  run base-otf ab_base "--alternate-corr" || exit 1
  run new-otf . "--alternate-corr" || exit 1
done
