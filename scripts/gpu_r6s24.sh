set -o pipefail
OUT=gpurun_out/r6s24
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 900 python -u scripts/tune_conv.py --merge --out $OUT/conv_tuning.json > $OUT/tune.log 2>&1 || { tail -30 $OUT/tune.log; exit 1; }
tail -3 $OUT/tune.log
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 30 > $OUT/b_old.$r.log 2>&1 || { tail -20 $OUT/b_old.$r.log; exit 1; }
tail -1 $OUT/b_old.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("old table", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
RS_CONV_TUNING_FILE=$OUT/conv_tuning.json timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 30 > $OUT/b_new.$r.log 2>&1 || { tail -20 $OUT/b_new.$r.log; exit 1; }
tail -1 $OUT/b_new.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("new table", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
done
