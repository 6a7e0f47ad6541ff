#!/bin/bash
# fp32 graphed inference with the per-shape layout tuner (ops/fp32conv.py) vs
# forced layouts: RAFT-small at the STIR size 512x640 and RAFT 1088x436.
set -o pipefail
mkdir -p gpurun_out/sp
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
run() { echo "$RS_FP32_LAYOUT $*" >> gpurun_out/sp/times.log; timeout -k 10 200 python scripts/infer_only.py "$@" >> gpurun_out/sp/times.log 2>&1; }
run --small --size 512 640 --graph --reps 30 --fp32 && RS_FP32_LAYOUT=nhwc run --small --size 512 640 --graph --reps 30 --fp32 && \
run --graph --reps 20 --fp32 && RS_FP32_LAYOUT=nhwc run --graph --reps 20 --fp32 && RS_FP32_LAYOUT=nchw run --graph --reps 20 --fp32
