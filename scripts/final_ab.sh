# same-box lines: HIP engine (RAFT, RAFT-small) and the stock-PyTorch A/B (both graphed for inference)
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/final/hip.log 2>&1 && tail -1 gpurun_out/final/hip.log && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --small > gpurun_out/final/small.log 2>&1 && tail -1 gpurun_out/final/small.log && \
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --reference-ops > gpurun_out/final/ref.log 2>&1 && tail -1 gpurun_out/final/ref.log
