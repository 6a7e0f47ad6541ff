"""Validation and benchmark-submission writers (reference evaluate.py:21-166).

Same functions, iteration counts and metric definitions:
  * ``validate_chairs(model, iters=24)``  -> {'chairs': mean EPE over all pixels}
  * ``validate_sintel(model, iters=32)``  -> {'clean': EPE, 'final': EPE} (+ 1/3/5 px
    printed), InputPadder('sintel')
  * ``validate_kitti(model, iters=24)``   -> {'kitti-epe': mean per-image EPE over
    valid px, 'kitti-f1': 100 * mean((epe > 3) & (epe/|gt| > 0.05))}, InputPadder('kitti')
  * ``create_sintel_submission(model, iters=32, warm_start=False, output_path=...)``
    (.flo per frame, optional forward-interpolated warm start)
  * ``create_kitti_submission(model, iters=24, output_path=...)`` (16-bit PNG)

Engine differences: on GPU each resolution is run through a cached hipGraph
of the whole forward (runtime.graph.GraphCache) -- one replay per pair --
and the per-pixel error statistics are reduced on the device (only a few
scalars per image cross to the host).  ``root=`` selects the dataset
location (reference: hard-coded ``datasets/``).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..data import datasets, frame_utils
from ..utils.geometry import forward_interpolate
from ..utils.padder import InputPadder


def _device(model):
    return next(model.parameters()).device


class _Runner:
    """model(image1, image2, iters, flow_init, test_mode=True), graphed on GPU."""

    def __init__(self, model, use_graph=True):
        self.model = model
        self.dev = _device(model)
        self.cache = None
        if use_graph and self.dev.type == "cuda" and os.environ.get("RAFT_STIR_NO_GRAPH") != "1":
            from ..runtime.graph import GraphCache
            self.cache = GraphCache(model)

    @torch.no_grad()
    def __call__(self, image1, image2, iters, flow_init=None):
        if self.cache is not None:
            lo, up = self.cache(image1, image2, iters=iters, flow_init=flow_init)
            return lo.clone(), up.clone()
        return self.model(image1, image2, iters=iters, flow_init=flow_init, test_mode=True)


def _to(dev, *xs):
    out = []
    for x in xs:
        x = x[None].to(dev, non_blocking=True)
        if dev.type == "cuda":
            x = x.contiguous(memory_format=torch.channels_last)
        out.append(x)
    return out


@torch.no_grad()
def create_sintel_submission(model, iters=32, warm_start=False, output_path="sintel_submission",
                             root="datasets/Sintel"):
    model.eval()
    run = _Runner(model)
    dev = run.dev
    for dstype in ["clean", "final"]:
        test_dataset = datasets.MpiSintel(split="test", aug_params=None, dstype=dstype, root=root)
        flow_prev, sequence_prev = None, None
        for test_id in range(len(test_dataset)):
            image1, image2, (sequence, frame) = test_dataset[test_id]
            if sequence != sequence_prev:
                flow_prev = None
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(*_to(dev, image1, image2))
            flow_low, flow_pr = run(image1, image2, iters, flow_init=flow_prev)
            flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
            if warm_start:
                flow_prev = forward_interpolate(flow_low[0])[None].to(dev)
            output_dir = os.path.join(output_path, dstype, sequence)
            os.makedirs(output_dir, exist_ok=True)
            frame_utils.writeFlow(os.path.join(output_dir, "frame%04d.flo" % (frame + 1)), flow)
            sequence_prev = sequence


@torch.no_grad()
def create_kitti_submission(model, iters=24, output_path="kitti_submission", root="datasets/KITTI"):
    model.eval()
    run = _Runner(model)
    test_dataset = datasets.KITTI(split="testing", aug_params=None, root=root)
    os.makedirs(output_path, exist_ok=True)
    for test_id in range(len(test_dataset)):
        image1, image2, (frame_id,) = test_dataset[test_id]
        padder = InputPadder(image1.shape, mode="kitti")
        image1, image2 = padder.pad(*_to(run.dev, image1, image2))
        _, flow_pr = run(image1, image2, iters)
        flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
        frame_utils.writeFlowKITTI(os.path.join(output_path, frame_id), flow)


@torch.no_grad()
def validate_chairs(model, iters=24, root="datasets/FlyingChairs_release/data",
                    split_file="chairs_split.txt"):
    model.eval()
    run = _Runner(model)
    val_dataset = datasets.FlyingChairs(split="validation", root=root, split_file=split_file)
    sum_epe, count = torch.zeros((), dtype=torch.float64, device=run.dev), 0
    for val_id in range(len(val_dataset)):
        image1, image2, flow_gt, _ = val_dataset[val_id]
        image1, image2 = _to(run.dev, image1, image2)
        _, flow_pr = run(image1, image2, iters)
        epe = torch.sum((flow_pr[0] - flow_gt.to(run.dev)) ** 2, dim=0).sqrt()
        sum_epe += epe.double().sum()
        count += epe.numel()
    if count == 0:
        # an empty/missing split must not report a perfect EPE of 0 (the
        # reference crashes in np.concatenate here; validate_sintel/kitti
        # likewise report nothing for absent data)
        raise FileNotFoundError(f"no FlyingChairs validation pairs under {root!r}")
    epe = float(sum_epe) / count
    print("Validation Chairs EPE: %f" % epe)
    return {"chairs": epe}


@torch.no_grad()
def validate_sintel(model, iters=32, root="datasets/Sintel"):
    model.eval()
    run = _Runner(model)
    results = {}
    for dstype in ["clean", "final"]:
        val_dataset = datasets.MpiSintel(split="training", dstype=dstype, root=root)
        acc = torch.zeros(4, dtype=torch.float64, device=run.dev)  # sum epe, <1, <3, <5
        count = 0
        for val_id in range(len(val_dataset)):
            image1, image2, flow_gt, _ = val_dataset[val_id]
            image1, image2 = _to(run.dev, image1, image2)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            _, flow_pr = run(image1, image2, iters)
            flow = padder.unpad(flow_pr[0])
            epe = torch.sum((flow - flow_gt.to(run.dev)) ** 2, dim=0).sqrt().reshape(-1).double()
            acc += torch.stack([epe.sum(), (epe < 1).sum(), (epe < 3).sum(), (epe < 5).sum()])
            count += epe.numel()
        if count == 0:
            print(f"Validation ({dstype}): no data under {root}")
            continue
        epe, px1, px3, px5 = (acc / count).tolist()
        print("Validation (%s) EPE: %f, 1px: %f, 3px: %f, 5px: %f" % (dstype, epe, px1, px3, px5))
        results[dstype] = epe
    return results


@torch.no_grad()
def validate_kitti(model, iters=24, root="datasets/KITTI"):
    model.eval()
    run = _Runner(model)
    val_dataset = datasets.KITTI(split="training", root=root)
    epe_list, out_sum, out_cnt = [], 0.0, 0
    for val_id in range(len(val_dataset)):
        image1, image2, flow_gt, valid_gt = val_dataset[val_id]
        image1, image2 = _to(run.dev, image1, image2)
        padder = InputPadder(image1.shape, mode="kitti")
        image1, image2 = padder.pad(image1, image2)
        _, flow_pr = run(image1, image2, iters)
        flow = padder.unpad(flow_pr[0])
        gt = flow_gt.to(run.dev)
        epe = torch.sum((flow - gt) ** 2, dim=0).sqrt().reshape(-1)
        mag = torch.sum(gt ** 2, dim=0).sqrt().reshape(-1)
        val = valid_gt.to(run.dev).reshape(-1) >= 0.5
        out = ((epe > 3.0) & ((epe / mag) > 0.05)).float()
        s = torch.stack([epe[val].double().mean(), out[val].double().sum(),
                         val.double().sum()]).tolist()
        epe_list.append(s[0])
        out_sum += s[1]
        out_cnt += int(s[2])
    if not epe_list:
        print(f"Validation KITTI: no data under {root}")
        return {}
    epe = float(np.mean(epe_list))
    f1 = 100.0 * out_sum / max(out_cnt, 1)
    print("Validation KITTI: %f, %f" % (epe, f1))
    return {"kitti-epe": epe, "kitti-f1": f1}


VALIDATORS = {"chairs": validate_chairs, "sintel": validate_sintel, "kitti": validate_kitti}
