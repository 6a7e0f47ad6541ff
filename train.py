#!/usr/bin/env python
"""RAFT training entry point (reference train.py CLI; see raft_stir_amd/train/trainer.py).

    python train.py --name raft-chairs --stage chairs --validation chairs --gpus 0 1 \
        --num_steps 100000 --batch_size 10 --lr 0.0004 --image_size 368 496 --wdecay 0.0001
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --stage synthetic ...
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from raft_stir_amd.train.trainer import main  # noqa: E402

if __name__ == "__main__":
    main()
