#!/usr/bin/env python
"""torch.profiler breakdown (aten op level, with input shapes) of one training
step and one inference forward -- finds the glue ops (copies, casts, cats)
around the HIP kernels.  Writes gpurun_out/torch_prof_{train,infer}.txt.

    python scripts/torch_prof.py [--batch 8] [--small] [--mode train|infer|both]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


GLUE = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::cat", "aten::scatter", "aten::gather", "aten::add",
        "aten::add_", "aten::mul", "aten::sub", "aten::rsqrt", "aten::sum", "aten::index", "aten::clone",
        "aten::contiguous", "aten::_to_copy", "aten::empty_like", "aten::zeros_like", "aten::index_select",
        "aten::copy", "aten::permute_copy", "aten::where", "aten::masked_fill", "aten::div", "aten::clamp", "aten::stack")


VENDOR = ("aten::convolution", "aten::convolution_backward", "aten::mm", "aten::bmm", "aten::addmm", "aten::matmul",
          "aten::baddbmm", "aten::_convolution")


class GlueTrace:
    """TorchDispatchMode that attributes every glue aten op (GLUE) to the
    innermost repo source line on the Python stack (the profiler's own stacks
    come back empty for ops issued from autograd.Function bodies on ROCm)."""

    def __init__(self, ops=GLUE):
        import traceback
        from torch.utils._python_dispatch import TorchDispatchMode
        agg = self.agg = {}

        class Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                name = "aten::" + func.__name__.split(".")[0]
                if name in ops:
                    where = "(no repo frame)"
                    for fr in reversed(traceback.extract_stack()):
                        if ("raft_stir_amd" in fr.filename or "/scripts/" in fr.filename) and \
                                "torch_prof.py" not in fr.filename:
                            where = f"{fr.filename.split('raft_stir_amd/')[-1]}:{fr.lineno} {fr.name}"
                            break
                    agg[(name, where)] = agg.get((name, where), 0) + 1
                return func(*args, **(kwargs or {}))
        self.mode = Mode()

    def write(self, path):
        with open(path, "w") as f:
            f.write(f"{'calls':>6}  op  @ innermost repo frame\n")
            for (name, where), c in sorted(self.agg.items(), key=lambda kv: -kv[1]):
                f.write(f"{c:6d}  {name}  @ {where}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--mode", default="both")
    ap.add_argument("--out", default="gpurun_out")
    ap.add_argument("--fp32", action="store_true", help="fp32 (no autocast), the reference's default precision")
    ap.add_argument("--vendor", action="store_true",
                    help="attribute the library-backed aten ops (convolution, mm, bmm, ...) instead of the glue ops")
    ap.add_argument("--stacks", action="store_true",
                    help="also attribute the glue ops (copy_, fill_, cat, scatter, ...) to Python source lines")
    a = ap.parse_args()
    from raft_stir_amd.config import make_args
    from raft_stir_amd.data.synthetic import make_batch
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RAFT(make_args(small=a.small, mixed_precision=not a.fp32)).to(dev).to(memory_format=torch.channels_last)
    os.makedirs(a.out, exist_ok=True)
    if a.mode in ("train", "both"):
        model.train()
        opt, sch = fetch_optimizer(argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000), model)
        i1, i2, fl, v = make_batch(a.batch, 368, 496, device=dev)

        def step():
            opt.zero_grad(set_to_none=True)
            loss, _ = sequence_loss(model(i1, i2, iters=12), fl, v, 0.8, sync_metrics=False)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
            opt.step()
            sch.step()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        if a.stacks or a.vendor:
            gt = GlueTrace(VENDOR if a.vendor else GLUE)
            with gt.mode:
                step()
            torch.cuda.synchronize()
            gt.write(os.path.join(a.out, "torch_vendor_train.txt" if a.vendor else "torch_glue_train.txt"))
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
            step()
            torch.cuda.synchronize()
        with open(os.path.join(a.out, "torch_prof_train.txt"), "w") as f:
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=80,
                                                                       max_name_column_width=60,
                                                                       max_shapes_column_width=90))
            f.write("\n\n")
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=60))
    if a.mode in ("infer", "both"):
        model.eval()
        from raft_stir_amd.utils.padder import InputPadder
        i1 = torch.rand(1, 3, 436, 1088, device=dev) * 255
        i2 = torch.rand(1, 3, 436, 1088, device=dev) * 255
        i1, i2 = InputPadder(i1.shape).pad(i1, i2)
        with torch.no_grad():
            for _ in range(3):
                model(i1, i2, iters=12, test_mode=True)
            torch.cuda.synchronize()
            if a.stacks:
                gt = GlueTrace()
                with gt.mode:
                    model(i1, i2, iters=12, test_mode=True)
                torch.cuda.synchronize()
                gt.write(os.path.join(a.out, "torch_glue_infer.txt"))
            with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
                model(i1, i2, iters=12, test_mode=True)
                torch.cuda.synchronize()
        with open(os.path.join(a.out, "torch_prof_infer.txt"), "w") as f:
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=80,
                                                                       max_name_column_width=60,
                                                                       max_shapes_column_width=90))
            f.write("\n\n")
            f.write(prof.key_averages().table(sort_by="cuda_time_total", row_limit=60, max_name_column_width=60))
    print("ok")


if __name__ == "__main__":
    main()
