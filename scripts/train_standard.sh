#!/bin/bash
# 4-stage RAFT schedule (reference train_standard.sh: Chairs -> Things -> Sintel -> KITTI,
# each stage warm-started from the previous one), on NGPU MI355X with DDP over RCCL.
# --batch_size is the GLOBAL batch; set DATA=<dir holding FlyingChairs_release/, Sintel/, ...>.
set -e
NGPU=${NGPU:-2}
DATA=${DATA:-datasets}
RUN="torchrun --standalone --nproc-per-node ${NGPU} train.py --data_root ${DATA} --resume auto"
mkdir -p checkpoints
$RUN --name raft-chairs --stage chairs --validation chairs --num_steps 100000 --batch_size 10 --lr 0.0004 --image_size 368 496 --wdecay 0.0001
$RUN --name raft-things --stage things --validation sintel --restore_ckpt checkpoints/raft-chairs.pth --num_steps 100000 --batch_size 6 --lr 0.000125 --image_size 400 720 --wdecay 0.0001
$RUN --name raft-sintel --stage sintel --validation sintel --restore_ckpt checkpoints/raft-things.pth --num_steps 100000 --batch_size 6 --lr 0.000125 --image_size 368 768 --wdecay 0.00001 --gamma=0.85
$RUN --name raft-kitti --stage kitti --validation kitti --restore_ckpt checkpoints/raft-sintel.pth --num_steps 50000 --batch_size 6 --lr 0.0001 --image_size 288 960 --wdecay 0.00001 --gamma=0.85
