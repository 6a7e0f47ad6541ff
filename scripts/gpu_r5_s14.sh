#!/bin/bash
# Round 5 session 14: in-house corr backward GEMMs, EPI_ADD_BF16 grad sink, retune with tiles 66-68, A/B.
set -o pipefail
OUT=gpurun_out/r5s14
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py -k "corr_volume_backward or pyr_grad_fold or allpairs" \
  tests/test_fused_gpu.py -k "add_bf16 or v3_epilogues" tests/test_enc_conv_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u scripts/bench_corr_bwd.py > $OUT/bench_corr_bwd.log 2>&1 || { tail -20 $OUT/bench_corr_bwd.log; exit 1; }
cat $OUT/bench_corr_bwd.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_before.json
timeout -k 10 900 python -u scripts/tune_conv.py --merge > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep -E "sum over" $OUT/tune.log
grep -cE "best t6[6-8]" $OUT/tune.log
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
for e in "RS_CONV_TUNING_FILE=$OUT/conv_tuning_before.json" "X=1" "RS_CONV_TUNING_FILE=$OUT/conv_tuning_before.json" "X=1"; do
  env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
  echo "[$e] $(tail -1 $OUT/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
