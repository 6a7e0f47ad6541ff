set -o pipefail
OUT=gpurun_out/r6s36
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp gpurun_out/conv_tuning_small.json $OUT/t.json
for r in 1 2; do
timeout -k 10 300 python bench.py --small --steps 60 --warmup 5 --infer-reps 40 > $OUT/b_old.$r.log 2>&1 || { tail -20 $OUT/b_old.$r.log; exit 1; }
tail -1 $OUT/b_old.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("old", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
RS_CONV_TUNING_FILE=$OUT/t.json timeout -k 10 300 python bench.py --small --steps 60 --warmup 5 --infer-reps 40 > $OUT/b_new.$r.log 2>&1 || { tail -20 $OUT/b_new.$r.log; exit 1; }
tail -1 $OUT/b_new.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("new", d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])'
done
