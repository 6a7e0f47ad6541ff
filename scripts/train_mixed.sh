#!/bin/bash
# Mixed-precision schedule (reference train_mixed.sh: 1 GPU, fp16 AMP); here bf16 autocast
# through the fused MI355X training engine, NGPU ranks (default 1).
set -e
NGPU=${NGPU:-1}
DATA=${DATA:-datasets}
RUN="torchrun --standalone --nproc-per-node ${NGPU} train.py --data_root ${DATA} --resume auto --mixed_precision"
mkdir -p checkpoints
$RUN --name raft-chairs --stage chairs --validation chairs --num_steps 120000 --batch_size 8 --lr 0.00025 --image_size 368 496 --wdecay 0.0001
$RUN --name raft-things --stage things --validation sintel --restore_ckpt checkpoints/raft-chairs.pth --num_steps 120000 --batch_size 5 --lr 0.0001 --image_size 400 720 --wdecay 0.0001
$RUN --name raft-sintel --stage sintel --validation sintel --restore_ckpt checkpoints/raft-things.pth --num_steps 120000 --batch_size 5 --lr 0.0001 --image_size 368 768 --wdecay 0.00001 --gamma=0.85
$RUN --name raft-kitti --stage kitti --validation kitti --restore_ckpt checkpoints/raft-sintel.pth --num_steps 50000 --batch_size 5 --lr 0.0001 --image_size 288 960 --wdecay 0.00001 --gamma=0.85
