#!/bin/bash
# gates for the new kernels (tiled OTF forward, conv tiles 51-53, fused
# clip+AdamW), conv retune with them, paired A/Bs, training profile, KITTI
# on-the-fly config, data feed
set -o pipefail
mkdir -p gpurun_out/s10
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  "tests/test_kernels_gpu.py::test_onthefly_tiled_forward" "tests/test_kernels_gpu.py::test_onthefly_corr_fwd_bwd" \
  "tests/test_kernels_gpu.py::test_onthefly_matches_allpairs" "tests/test_fused_gpu.py::test_conv_v2_tiles_vs_conv2d" \
  tests/test_optim_gpu.py > gpurun_out/s10/gates.log 2>&1; rc=$?
tail -15 gpurun_out/s10/gates.log
if [[ $rc -ne 0 ]]; then exit $rc; fi
cp raft_stir_amd/conv_tuning.json gpurun_out/s10/conv_tuning_before.json
timeout -k 10 600 python -u scripts/tune_conv.py --merge > gpurun_out/s10/tune.log 2>&1 || { tail -20 gpurun_out/s10/tune.log; exit 1; }
grep -E "train|infer|sum over" gpurun_out/s10/tune.log | tail -45
cp raft_stir_amd/conv_tuning.json gpurun_out/s10/conv_tuning.json
for e in "X=1" "RS_FUSED_ADAMW=0" "RS_NORM_RED_BLOCKS=2048" "RS_STEM=1" "X=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s10/ab.log 2>&1 || { tail -20 gpurun_out/s10/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s10/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/s10/bench.log 2>&1 && tail -1 gpurun_out/s10/bench.log
timeout -k 10 300 python scripts/bench_configs.py --only 4 > gpurun_out/s10/kitti.log 2>&1 && tail -2 gpurun_out/s10/kitti.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/proft -o t -- python3 bench.py --steps 10 --warmup 3 --no-infer > gpurun_out/s10/prof_train.log 2>&1 || { tail -5 gpurun_out/s10/prof_train.log; exit 1; }
find /tmp/proft -name "*kernel_stats.csv" -exec cp {} gpurun_out/s10/train_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s10/train_kernel_stats.csv 13 2>&1 | head -30 || true
timeout -k 10 240 python scripts/bench_dataloader.py --workers 4 --batches 40 2>&1 | tail -1 | tee -a gpurun_out/s10/feed.jsonl
