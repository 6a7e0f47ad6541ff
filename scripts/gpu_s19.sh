#!/bin/bash
# tiled on-the-fly correlation backward (gate + A/B), stream priorities,
# residual-sink A/B, on-the-fly training benches and profile
set -o pipefail
mkdir -p gpurun_out/s19
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_onthefly_tiled_backward" "tests/test_kernels_gpu.py::test_onthefly_corr_fwd_bwd" \
  "tests/test_kernels_gpu.py::test_onthefly_tiled_forward" > gpurun_out/s19/gates.log 2>&1; rc=$?
tail -15 gpurun_out/s19/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
for e in "X=1 --small --alternate-corr" "RS_OTF_TILE_BWD=0 --small --alternate-corr" "X=1 --alternate-corr" "RS_OTF_TILE_BWD=0 --alternate-corr" "X=1 --small"; do
  set -- $e
  env $1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-infer "${@:2}" > gpurun_out/s19/otf.log 2>&1 || { tail -20 gpurun_out/s19/otf.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s19/otf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/potf -o t -- python3 bench.py --steps 3 --warmup 2 --no-infer --small --alternate-corr > gpurun_out/s19/prof_otf.log 2>&1 || { tail -5 gpurun_out/s19/prof_otf.log; exit 1; }
find /tmp/potf -name "*kernel_stats.csv" -exec cp {} gpurun_out/s19/small_otf_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s19/small_otf_kernel_stats.csv 5 2>&1 | head -16 || true
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for e in "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1" "RS_RES_SINK=0" "X=1" "RS_WGRAD_PRIO=1" "RS_SIDE_PRIO=-1" "RS_RES_SINK=0"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s19/ab.log 2>&1 || { tail -20 gpurun_out/s19/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s19/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
