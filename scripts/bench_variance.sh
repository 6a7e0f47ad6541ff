# bench.py repeated on one box: default flags and the short form (run-to-run / warm-up spread)
mkdir -p gpurun_out/var
for i in 1 2; do
  timeout -k 10 200 python bench.py > gpurun_out/var/def_$i.log 2>&1 || exit 1
  echo "default   $(tail -1 gpurun_out/var/def_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/var/short_$i.log 2>&1 || exit 1
  echo "s10 w3    $(tail -1 gpurun_out/var/short_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["inference"]["fps"])')"
done
