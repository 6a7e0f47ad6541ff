set -o pipefail
OUT=gpurun_out/r6s40
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2; do
for v in 0 1; do
HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 40 > $OUT/b$v.$r.log 2>&1 || { tail -20 $OUT/b$v.$r.log; exit 1; }
echo "kernarg=$v run $r: $(tail -1 $OUT/b$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])')"
HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --small --eager --steps 30 --warmup 5 --infer-reps 40 > $OUT/s$v.$r.log 2>&1 || { tail -20 $OUT/s$v.$r.log; exit 1; }
echo "kernarg=$v small-eager run $r: $(tail -1 $OUT/s$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["ms_per_pair"])')"
done
done
