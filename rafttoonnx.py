#!/usr/bin/env python
"""STIR export (reference rafttoonnx.py): RAFT-small point tracker ->
TorchScript ``raft_pointtrackSTIR.pt`` (+ ``raft_pointtrackSTIR.onnx`` when the
onnx package is installed), plus the bare-model exports
``raftsmall.onnx`` (demo-frame shape) and ``raftsmall_STIR.onnx`` (1x3x512x640).

Defaults match the reference's hard-coded values (models/raft-small.pth,
demo-frames, RAFT-small), but unlike the reference the CLI flags are honoured
(defect B12) and the export images are in [0, 255].  A missing checkpoint is
an error unless ``--random_init`` is given (then random-init weights).
"""
import argparse
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from raft_stir_amd.cli_common import add_model_args, load_image, load_model  # noqa: E402
from raft_stir_amd.export.pointtrack import (NUMITERS, POINTCOUNT, RaftPointTrack, _FlowOnly,  # noqa: E402
                                             _reference_mode, export_onnx, export_pointtrack,
                                             export_torchscript, onnx_available)
from raft_stir_amd.utils.padder import InputPadder  # noqa: E402


def _torchscript_fallback(module, inputs, path, device):
    """No onnx package: the same graph as TorchScript, reloaded and checked
    against eager at the reference's ONNX tolerance (atol = rtol = 1e-2,
    reference rafttoonnx.py:88; measured differences are ~1e-5)."""
    module.eval()
    with torch.no_grad(), _reference_mode():
        traced = torch.jit.trace(module, inputs, check_trace=False)
        traced.save(path)
        want, got = module(*inputs), torch.jit.load(path, map_location=device)(*inputs)
    err = max((w - g).abs().max().item() for w, g in zip(want, got))
    for w, g in zip(want, got):
        if not torch.allclose(g, w, atol=1e-2, rtol=1e-2):
            raise AssertionError(f"{os.path.basename(path)} parity failed: max|diff|={err}")
    print(f"onnx not installed: wrote {path} (TorchScript, max|diff| vs eager {err:.2e})")
    return path


def testconvertmodel(args, device):
    """Bare model on padded demo frames -> raftsmall.onnx (reference :49-92)."""
    images = sorted(glob.glob(os.path.join(args.path, "*.png")) + glob.glob(os.path.join(args.path, "*.jpg")))
    if len(images) < 2:
        raise FileNotFoundError(f"testconvertmodel: need >= 2 frames in {args.path!r} "
                                "(demo-frames/ ships with the repo: scripts/make_demo_frames.py)")
    model = load_model(args, device)
    image1, image2 = load_image(images[0], device), load_image(images[1], device)
    image1, image2 = InputPadder(image1.shape).pad(image1, image2)
    module = _FlowOnly(model, NUMITERS)
    if onnx_available():
        return export_onnx(module, (image1, image2), os.path.join(args.out, "raftsmall.onnx"),
                           ["image1", "image2"], ["flow_low", "flow_up"])
    return _torchscript_fallback(module, (image1, image2), os.path.join(args.out, "raftsmall.pt"), device)


def convertmodeldirect(args, device, size=(512, 640)):
    """Bare model on 1x3x512x640 (the STIR frame shape) -> raftsmall_STIR.onnx
    (reference :94-118); without onnx, raftsmall_STIR.pt (TorchScript) with
    the same parity check."""
    model = load_model(args, device)
    g = torch.Generator().manual_seed(0)
    image1 = (torch.rand(1, 3, *size, generator=g) * 255).to(device)
    image2 = (torch.rand(1, 3, *size, generator=g) * 255).to(device)
    module = _FlowOnly(model, NUMITERS)
    if onnx_available():
        return export_onnx(module, (image1, image2), os.path.join(args.out, "raftsmall_STIR.onnx"),
                           ["image1", "image2"], ["flow_low", "flow_up"])
    return _torchscript_fallback(module, (image1, image2), os.path.join(args.out, "raftsmall_STIR.pt"), device)


def convertmodelpointtrack(args, device):
    """STIR tracker -> raft_pointtrackSTIR.{pt,onnx} (reference :156-223)."""
    model = load_model(args, device)
    return export_pointtrack(model, os.path.join(args.out, "raft_pointtrackSTIR"), size=(512, 640),
                             npoints=POINTCOUNT, device=device)


if __name__ == "__main__":
    parser = argparse.ArgumentParser()
    add_model_args(parser)
    parser.add_argument("--model", default="models/raft-small.pth", help="restore checkpoint")
    parser.add_argument("--path", default="demo-frames", help="frames for the demo-shape export")
    parser.add_argument("--small", action=argparse.BooleanOptionalAction, default=True)
    parser.add_argument("--mixed_precision", action="store_true", help="ignored for export (fp32)")
    parser.add_argument("--alternate_corr", action="store_true")
    parser.add_argument("--device", default="cpu", help="export device (graphs hold only standard ops)")
    parser.add_argument("--out", default=".")
    args = parser.parse_args()
    args.mixed_precision = False
    dev = torch.device(args.device)
    os.makedirs(args.out, exist_ok=True)
    testconvertmodel(args, dev)
    convertmodeldirect(args, dev)
    print(convertmodelpointtrack(args, dev))
