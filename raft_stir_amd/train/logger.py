"""Training logger (reference train.py:89-133 ``Logger``).

Same observable behaviour: running sums of the step metrics, and every
``sum_freq`` (100) steps a ``[step, lr] metric...`` line on stdout plus one
scalar per metric (names ``epe``, ``1px``, ``3px``, ``5px``; validation
``chairs``/``clean``/``final``/``kitti-epe``/``kitti-f1`` via
:meth:`write_dict`).

Differences:
  * metrics are pushed as device tensors and summed on device; they are
    materialised (one host sync, one all-reduce across ranks) only at the
    print boundary, never per step (the reference's four ``.item()`` calls per
    step stall the launch queue);
  * throughput (pairs/s), ms/step and peak HBM are logged alongside;
  * scalars go to TensorBoard when it is importable and ALWAYS to a JSONL
    file (``log_dir/metrics.jsonl``);
  * :meth:`close` is safe when fewer than ``sum_freq`` steps ran (reference
    defect B11).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import torch


class Logger:
    def __init__(self, model=None, scheduler=None, sum_freq: int = 100, log_dir: Optional[str] = None,
                 rank: int = 0, pairs_per_step: int = 0, reduce_fn=None, start_step: int = 0):
        self.model = model
        self.scheduler = scheduler
        self.sum_freq = sum_freq
        self.total_steps = start_step
        self.running_loss: Dict[str, torch.Tensor] = {}
        self.rank = rank
        self.log_dir = log_dir
        self.writer = None
        self.pairs_per_step = pairs_per_step
        self.reduce_fn = reduce_fn
        self._t0 = time.perf_counter()
        self._n = 0
        self._jsonl = None
        self.history = []

    # ------------------------------------------------------------ outputs
    def _open(self):
        if self.rank != 0:
            return
        if self.log_dir and self._jsonl is None:
            os.makedirs(self.log_dir, exist_ok=True)
            self._jsonl = open(os.path.join(self.log_dir, "metrics.jsonl"), "a")
        if self.writer is None:
            try:
                from torch.utils.tensorboard import SummaryWriter
                self.writer = SummaryWriter(self.log_dir) if self.log_dir else SummaryWriter()
            except Exception:
                self.writer = False

    def _emit(self, step: int, scalars: Dict[str, float], kind: str):
        if self.rank != 0:
            return
        self._open()
        rec = {"step": step, "kind": kind, **scalars}
        self.history.append(rec)
        if self._jsonl:
            self._jsonl.write(json.dumps(rec) + "\n")
            self._jsonl.flush()
        if self.writer:
            for k, v in scalars.items():
                self.writer.add_scalar(k, v, step)

    # ------------------------------------------------------------ API
    def _print_training_status(self):
        n = max(self._n, 1)
        keys = sorted(self.running_loss)
        vals = torch.stack([self.running_loss[k].detach().double().reshape(()) for k in keys])
        if self.reduce_fn is not None:
            vals = self.reduce_fn(vals)
        vals = (vals / n).tolist()
        metrics = dict(zip(keys, vals))
        dt = time.perf_counter() - self._t0
        lr = self.scheduler.get_last_lr()[0] if self.scheduler is not None else 0.0
        extra = {"ms_per_step": 1000.0 * dt / n}
        if self.pairs_per_step:
            extra["pairs_per_s"] = self.pairs_per_step * n / dt
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            extra["peak_hbm_gb"] = torch.cuda.max_memory_allocated() / 1e9
        if self.rank == 0:
            status = "[{:6d}, {:10.7f}] ".format(self.total_steps + 1, lr)
            status += ("{:10.4f}, " * len(vals)).format(*vals)
            status += " | " + ", ".join(f"{k} {v:.2f}" for k, v in extra.items())
            print(status, flush=True)
        self._emit(self.total_steps, {**metrics, "lr": lr, **extra}, "train")
        self.running_loss = {}
        self._n = 0
        self._t0 = time.perf_counter()

    def push(self, metrics: Dict):
        self.total_steps += 1
        for k, v in metrics.items():
            t = v.detach() if isinstance(v, torch.Tensor) else torch.tensor(float(v))
            t = t.double() if t.device.type == "cpu" else t.float()
            self.running_loss[k] = self.running_loss[k] + t if k in self.running_loss else t
        self._n += 1
        if self.total_steps % self.sum_freq == self.sum_freq - 1:
            self._print_training_status()

    def write_dict(self, results: Dict[str, float]):
        self._emit(self.total_steps, {k: float(v) for k, v in results.items()}, "val")

    def close(self):
        if self.writer:
            self.writer.close()
        if self._jsonl:
            self._jsonl.close()
            self._jsonl = None
