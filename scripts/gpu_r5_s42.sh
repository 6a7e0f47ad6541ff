#!/bin/bash
# Round 5 session 42-43: OTF MFMA backward (row-major staging + tr16 reads; 32-channel f2 chunks) (tests, microbench, OTF training).
set -o pipefail
OUT=gpurun_out/r5s${SESSION:-42}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_determinism_gpu.py tests/test_fused_train_gpu.py -k "onthefly or otf" > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python scripts/bench_otf_bwd.py > $OUT/otf_bwd.log 2>&1 || { tail -20 $OUT/otf_bwd.log; exit 1; }
cat $OUT/otf_bwd.log
for a in "--small --alternate-corr" "--alternate-corr"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $a > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  echo "[$a] $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $OUT/ab.txt
done
