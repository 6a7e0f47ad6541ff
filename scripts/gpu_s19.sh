#!/bin/bash
# stream priorities: encoder backward vs the deferred weight gradients
set -o pipefail
mkdir -p gpurun_out/s19
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for e in "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1" "RS_RES_SINK=0" "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1" "RS_RES_SINK=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s19/ab.log 2>&1 || { tail -20 gpurun_out/s19/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s19/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
for args in "--small --alternate-corr" "--small" "--alternate-corr"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer $args > gpurun_out/s19/otf.log 2>&1 || { tail -20 gpurun_out/s19/otf.log; exit 1; }
  echo "[$args] $(tail -1 gpurun_out/s19/otf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/potf -o t -- python3 bench.py --steps 3 --warmup 2 --no-infer --small --alternate-corr > gpurun_out/s19/prof_otf.log 2>&1 || { tail -5 gpurun_out/s19/prof_otf.log; exit 1; }
find /tmp/potf -name "*kernel_stats.csv" -exec cp {} gpurun_out/s19/small_otf_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s19/small_otf_kernel_stats.csv 5 2>&1 | head -16 || true
timeout -k 10 900 python -u scripts/fidelity_ensemble.py --seeds 3 > gpurun_out/s19/fid_ens.log 2>&1; grep -v "amdgpu\|Warning\|sched.step" gpurun_out/s19/fid_ens.log
