set -o pipefail
OUT=gpurun_out/r6s28
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cp raft_stir_amd/conv_tuning.json $OUT/conv_tuning.json
timeout -k 10 900 python -u scripts/tune_conv.py --f32 --merge --out $OUT/conv_tuning.json > $OUT/tune_f32.log 2>&1 || { tail -30 $OUT/tune_f32.log; exit 1; }
tail -2 $OUT/tune_f32.log
for r in 1 2; do
timeout -k 10 300 python scripts/infer_only.py --fp32 --graph --reps 30 > $OUT/inf_old.$r.log 2>&1 || { tail -5 $OUT/inf_old.$r.log; exit 1; }
echo "old: $(tail -1 $OUT/inf_old.$r.log)"
RS_CONV_TUNING_FILE=$OUT/conv_tuning.json timeout -k 10 300 python scripts/infer_only.py --fp32 --graph --reps 30 > $OUT/inf_new.$r.log 2>&1 || { tail -5 $OUT/inf_new.$r.log; exit 1; }
echo "new: $(tail -1 $OUT/inf_new.$r.log)"
done
