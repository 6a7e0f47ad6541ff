set -o pipefail
OUT=gpurun_out/r6s35
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python scripts/host_profile.py --steps 20 > $OUT/host.log 2>&1 || { tail -20 $OUT/host.log; exit 1; }
head -3 $OUT/host.log
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-infer > $OUT/b_eager.$r.log 2>&1 || { tail -20 $OUT/b_eager.$r.log; exit 1; }
tail -1 $OUT/b_eager.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("eager", d["value"], d["ms_per_step"])'
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-infer --train-graph > $OUT/b_graph.$r.log 2>&1 || { tail -20 $OUT/b_graph.$r.log; exit 1; }
tail -1 $OUT/b_graph.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("graph", d["value"], d["ms_per_step"])'
done
