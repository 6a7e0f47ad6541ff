#!/bin/bash
# conv retune with the MW=2 tiles (48-50), feed bench on the new host ops,
# paired A/B of the norm reduction grid size
set -o pipefail
mkdir -p gpurun_out/s9
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread "tests/test_fused_gpu.py::test_conv_v2_tiles_vs_conv2d" > gpurun_out/s9/v2tiles.log 2>&1 || { tail -30 gpurun_out/s9/v2tiles.log; exit 1; }
tail -2 gpurun_out/s9/v2tiles.log
for w in 4 8; do
  timeout -k 10 240 python scripts/bench_dataloader.py --workers $w --batches 40 2>&1 | tail -1 | tee -a gpurun_out/s9/feed.jsonl || exit 1
done
cp raft_stir_amd/conv_tuning.json gpurun_out/s9/conv_tuning_before.json
timeout -k 10 500 python -u scripts/tune_conv.py --merge > gpurun_out/s9/tune_train.log 2>&1 || { tail -20 gpurun_out/s9/tune_train.log; exit 1; }
tail -3 gpurun_out/s9/tune_train.log
cp raft_stir_amd/conv_tuning.json gpurun_out/s9/conv_tuning.json
for rep in 1 2; do for e in "X=1" "RS_NORM_RED_BLOCKS=2048" "RS_NORM_RED_BLOCKS=1024" "RS_STEM=1"; do
  env $e timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-infer > gpurun_out/s9/ab.log 2>&1 || { tail -20 gpurun_out/s9/ab.log; exit 1; }
  echo "[$e] $(tail -1 gpurun_out/s9/ab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["final_loss"])')"
done; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profk -o t -- python3 scripts/bench_configs.py --only 4 > gpurun_out/s9/prof_kitti.log 2>&1 || { tail -5 gpurun_out/s9/prof_kitti.log; exit 1; }
find /tmp/profk -name "*kernel_stats.csv" -exec cp {} gpurun_out/s9/kitti_kernel_stats.csv \;
head -25 gpurun_out/s9/kitti_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/proft -o t -- python3 bench.py --steps 10 --warmup 3 --no-infer > gpurun_out/s9/prof_train.log 2>&1 || { tail -5 gpurun_out/s9/prof_train.log; exit 1; }
find /tmp/proft -name "*kernel_stats.csv" -exec cp {} gpurun_out/s9/train_kernel_stats.csv \;
python3 scripts/prof_categories.py gpurun_out/s9/train_kernel_stats.csv 13 2>&1 | head -40 || true
