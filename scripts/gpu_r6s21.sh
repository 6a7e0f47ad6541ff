set -o pipefail
OUT=gpurun_out/r6s21
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2; do
for v in 0 1; do
RS_V3F=$v timeout -k 10 300 python bench.py --fp32 --steps 12 --warmup 3 --no-infer > $OUT/b_fp32_v3f$v.$r.log 2>&1 || { tail -20 $OUT/b_fp32_v3f$v.$r.log; exit 1; }
echo "v3f=$v run $r: $(tail -1 $OUT/b_fp32_v3f$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 900 python -u scripts/tune_conv.py --f32 --merge --out $OUT/conv_tuning.json > $OUT/tune_f32.log 2>&1 || { tail -30 $OUT/tune_f32.log; exit 1; }
tail -5 $OUT/tune_f32.log
