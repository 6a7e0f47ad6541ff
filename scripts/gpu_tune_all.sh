#!/bin/bash
# Retune every conv call table (training, RAFT / RAFT-small / STIR / KITTI /
# Sintel-1024 inference) with the current tile set, then a same-box A/B of the
# new table against the old one.  TEST=1: run tests/test_fused_gpu.py first.
set -o pipefail
OUT=${OUT:-gpurun_out/tune_all}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
if [[ -n "$TEST" ]]; then
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fused_gpu.py > $OUT/pytest.log 2>&1 || { echo PYTEST FAILED; tail -40 $OUT/pytest.log; exit 1; }
  tail -1 $OUT/pytest.log
fi
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning_old.json
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
T="timeout -k 10 600 python scripts/tune_conv.py --merge --out $OUT/conv_tuning.json"
$T > $OUT/tune_train.log 2>&1 || { tail -20 $OUT/tune_train.log; exit 1; }
$T --small --infer-only > $OUT/tune_small.log 2>&1 || { tail -20 $OUT/tune_small.log; exit 1; }
$T --small --infer-only --infer-size 512 640 > $OUT/tune_stir.log 2>&1 || { tail -20 $OUT/tune_stir.log; exit 1; }
$T --infer-only --infer-size 375 1242 > $OUT/tune_kitti.log 2>&1 || { tail -20 $OUT/tune_kitti.log; exit 1; }
$T --infer-only --infer-size 436 1024 > $OUT/tune_sintel1024.log 2>&1 || { tail -20 $OUT/tune_sintel1024.log; exit 1; }
python - $OUT/conv_tuning_old.json $OUT/conv_tuning.json <<'PY' | tee $OUT/diff.txt
import json, sys
a = json.load(open(sys.argv[1]))["tiles"]; b = json.load(open(sys.argv[2]))["tiles"]
for k in sorted(set(a) | set(b)):
    if a.get(k) != b.get(k):
        print(k, a.get(k), "->", b.get(k))
PY
for t in new old new old; do
  if [[ $t == new ]]; then cp $OUT/conv_tuning.json raft_stir_amd/conv_tuning.json; else cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json; fi
  timeout -k 10 400 python bench.py --steps 30 --warmup 5 --infer-reps 50 > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
  timeout -k 10 300 python scripts/infer_only.py --small --graph --reps 50 > $OUT/i.log 2>&1 || { tail -20 $OUT/i.log; exit 1; }
  timeout -k 10 300 python scripts/stir_only.py --bf16 --reps 50 > $OUT/s.log 2>&1 || { tail -20 $OUT/s.log; exit 1; }
  echo "[$t] $(tail -1 $OUT/b.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], (d.get("inference") or {}).get("fps"))') | $(tail -1 $OUT/i.log) | $(tail -1 $OUT/s.log)" | tee -a $OUT/ab.txt
done
cp $OUT/conv_tuning_old.json raft_stir_amd/conv_tuning.json
