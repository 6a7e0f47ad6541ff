#!/usr/bin/env python
"""Evaluation entry point (reference evaluate.py CLI).

    python evaluate.py --model models/raft-things.pth --dataset sintel [--mixed_precision]
    python evaluate.py --model ... --dataset kitti --submission   # write KITTI submission
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from raft_stir_amd.cli_common import add_model_args, load_model  # noqa: E402
from raft_stir_amd.eval.evaluate import (  # noqa: E402,F401
    create_kitti_submission, create_sintel_submission, validate_chairs, validate_kitti,
    validate_sintel)


def main(argv=None):
    parser = argparse.ArgumentParser()
    add_model_args(parser)
    parser.add_argument("--model", help="restore checkpoint")
    parser.add_argument("--dataset", help="dataset for evaluation: chairs | sintel | kitti")
    parser.add_argument("--small", action="store_true", help="use small model")
    parser.add_argument("--mixed_precision", action="store_true", help="bf16 autocast")
    parser.add_argument("--alternate_corr", action="store_true",
                        help="use efficient (on-the-fly) correlation implementation")
    parser.add_argument("--data_root", default="datasets")
    parser.add_argument("--iters", type=int, default=None, help="override the per-dataset default")
    parser.add_argument("--submission", action="store_true", help="write a benchmark submission")
    parser.add_argument("--warm_start", action="store_true", help="Sintel submission warm start")
    parser.add_argument("--output_path", default=None)
    args = parser.parse_args(argv)

    model = load_model(args)
    kw = {} if args.iters is None else {"iters": args.iters}
    root = args.data_root
    with torch.no_grad():
        if args.submission:
            if args.dataset == "sintel":
                create_sintel_submission(model, warm_start=args.warm_start, root=os.path.join(root, "Sintel"),
                                         output_path=args.output_path or "sintel_submission", **kw)
            elif args.dataset == "kitti":
                create_kitti_submission(model, root=os.path.join(root, "KITTI"),
                                        output_path=args.output_path or "kitti_submission", **kw)
            return None
        if args.dataset == "chairs":
            return validate_chairs(model, root=os.path.join(root, "FlyingChairs_release/data"), **kw)
        if args.dataset == "sintel":
            return validate_sintel(model, root=os.path.join(root, "Sintel"), **kw)
        if args.dataset == "kitti":
            return validate_kitti(model, root=os.path.join(root, "KITTI"), **kw)
    raise SystemExit(f"unknown dataset {args.dataset!r}")


if __name__ == "__main__":
    main()
