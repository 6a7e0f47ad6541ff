#!/usr/bin/env python
"""Demo (reference demo.py): flow for every consecutive frame pair of a folder.

    python demo.py --model models/raft-things.pth --path demo-frames [--out demo-out]

Writes ``<out>/<frame>_flow.png`` (image above its Middlebury-coloured flow,
reference viz layout) and ``.flo`` files instead of opening a cv2 window
(no display/cv2 on MI355X servers).  The reference's per-pair ONNX
re-export, ``breakpoint()`` and broken viz call (defect B9) are not
reproduced; export lives in rafttoonnx.py.
"""
import argparse
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from raft_stir_amd.cli_common import add_model_args, default_device, load_image, load_model  # noqa: E402
from raft_stir_amd.data import frame_utils  # noqa: E402
from raft_stir_amd.utils import flow_viz  # noqa: E402
from raft_stir_amd.utils.padder import InputPadder  # noqa: E402


def viz(img, flo, out_file):
    img = img[0].permute(1, 2, 0).cpu().numpy()
    flo = flow_viz.flow_to_image(flo[0].permute(1, 2, 0).cpu().numpy())
    Image.fromarray(np.concatenate([img, flo], axis=0).astype(np.uint8)).save(out_file)


def demo(args):
    dev = default_device()
    model = load_model(args, dev)
    images = sorted(glob.glob(os.path.join(args.path, "*.png")) + glob.glob(os.path.join(args.path, "*.jpg")))
    os.makedirs(args.out, exist_ok=True)
    outs = []
    with torch.no_grad():
        for imfile1, imfile2 in zip(images[:-1], images[1:]):
            image1 = load_image(imfile1, dev)
            image2 = load_image(imfile2, dev)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            flow_low, flow_up = model(image1, image2, iters=args.iters, test_mode=True)
            flow_up = padder.unpad(flow_up)
            stem = os.path.splitext(os.path.basename(imfile1))[0]
            viz(padder.unpad(image1), flow_up, os.path.join(args.out, stem + "_flow.png"))
            frame_utils.writeFlow(os.path.join(args.out, stem + ".flo"),
                                  flow_up[0].permute(1, 2, 0).cpu().numpy())
            outs.append(stem)
    print(f"wrote {len(outs)} flow fields to {args.out}")
    return outs


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    add_model_args(parser)
    parser.add_argument("--model", help="restore checkpoint")
    parser.add_argument("--path", help="dataset for evaluation")
    parser.add_argument("--small", action="store_true", help="use small model")
    parser.add_argument("--mixed_precision", action="store_true", help="use mixed precision")
    parser.add_argument("--alternate_corr", action="store_true", help="use efficent correlation implementation")
    parser.add_argument("--iters", type=int, default=20)
    parser.add_argument("--out", default="demo-out")
    demo(parser.parse_args())
