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


def load_model(args, device=None, eval_mode=True):
    """RAFT(args) + weights from ``args.model`` (reference or engine layout,
    ``module.``-prefixed or not); random init (with a warning) if the file
    does not exist -- there is no network to download pretrained weights."""
    device = device or default_device()
    model = RAFT(make_args(small=getattr(args, "small", False),
                           mixed_precision=getattr(args, "mixed_precision", False),
                           alternate_corr=getattr(args, "alternate_corr", False)))
    path = getattr(args, "model", None)
    if path and os.path.exists(path):
        ckpt.load_weights(model, path, strict=False)
    elif path:
        print(f"warning: {path} not found; using random-init weights")
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
