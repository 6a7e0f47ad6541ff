set -o pipefail
mkdir -p gpurun_out/t5
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_segments or gru" > gpurun_out/t5/pytest.log 2>&1 || { tail -30 gpurun_out/t5/pytest.log; exit 1; }
tail -2 gpurun_out/t5/pytest.log
cp raft_stir_amd/conv_tuning.json gpurun_out/t5/conv_tuning.json
timeout -k 10 600 python scripts/tune_conv.py --merge --out gpurun_out/t5/conv_tuning.json > gpurun_out/t5/tune.log 2>&1 || { tail -30 gpurun_out/t5/tune.log; exit 1; }
tail -3 gpurun_out/t5/tune.log
cp gpurun_out/t5/conv_tuning.json raft_stir_amd/conv_tuning.json
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --infer-reps 50 > gpurun_out/t5/bench.log 2>&1 || { tail -30 gpurun_out/t5/bench.log; exit 1; }
tail -1 gpurun_out/t5/bench.log
