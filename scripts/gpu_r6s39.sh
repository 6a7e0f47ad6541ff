set -o pipefail
OUT=gpurun_out/r6s39
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for r in 1 2; do
for v in 300000 400000 1000000; do
RS_HALO_MIN_P=$v timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-infer > $OUT/b$v.$r.log 2>&1 || { tail -20 $OUT/b$v.$r.log; exit 1; }
echo "halo_min_p=$v run $r: $(tail -1 $OUT/b$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
done
