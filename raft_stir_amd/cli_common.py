"""Helpers shared by the root CLI scripts (evaluate.py, demo.py, rafttoonnx.py)."""
from __future__ import annotations

import os

import numpy as np
import torch
from PIL import Image

from .config import make_args
from .models import RAFT
from .train import checkpoint as ckpt


def default_device() -> torch.device:
    return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")


def add_model_args(parser):
    """--random_init: the explicit opt-in for running without a checkpoint."""
    parser.add_argument("--random_init", action="store_true",
                        help="run with random-init weights when --model is absent (no checkpoint)")
    return parser


def load_model(args, device=None, eval_mode=True):
    """RAFT(args) + weights from ``args.model`` (reference or engine layout,
    ``module.``-prefixed or not), loaded STRICTLY like the reference CLIs
    (/root/reference/evaluate.py:173, demo.py:50).  A missing checkpoint is
    an error unless ``args.random_init`` opts into random-init weights (there
    is no network to download pretrained ones) -- a typo in --model must not
    silently produce evaluations or exports from random weights."""
    device = device or default_device()
    model = RAFT(make_args(small=getattr(args, "small", False),
                           mixed_precision=getattr(args, "mixed_precision", False),
                           alternate_corr=getattr(args, "alternate_corr", False)))
    path = getattr(args, "model", None)
    if path and os.path.exists(path):
        ckpt.load_weights(model, path, strict=True)
    elif getattr(args, "random_init", False):
        print(f"--random_init: using random-init weights ({path or 'no --model'})")
    else:
        raise FileNotFoundError(f"checkpoint {path!r} not found (pass --random_init to run without one)")
    model.to(device)
    if device.type == "cuda":
        model.to(memory_format=torch.channels_last)
    return model.eval() if eval_mode else model


def load_image(imfile, device):
    img = np.array(Image.open(imfile)).astype(np.uint8)
    if img.ndim == 2:
        img = np.tile(img[..., None], (1, 1, 3))
    img = torch.from_numpy(img[..., :3]).permute(2, 0, 1).float()
    return img[None].to(device)
