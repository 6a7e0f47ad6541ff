"""Process-group setup and data parallelism over RCCL (xGMI) / gloo.

Replaces the reference's single-process ``nn.DataParallel`` (train.py:138;
broadcast of all parameters every forward, gather of 12 full-resolution
predictions to GPU0, reduce of gradients to GPU0 -- SURVEY §2.5) with one
process per GPU:

* ``torch.distributed`` backend ``nccl`` (= RCCL on ROCm) for GPUs, ``gloo``
  for CPU ranks (tests);
* gradients all-reduced in buckets by DDP hooks *during* backward on DDP's
  communication stream, overlapping the unrolled 12-iteration backward.
  RAFT's 21 MB of fp32 gradients are split into ~5 MB buckets so the first
  all-reduces start while the encoder backward is still running; on an
  8 x MI355X node a ring over the 7 xGMI links moves ~37 MB per rank per step,
  well under 1 % of a training step;
* the loss is computed on each rank (no prediction gather at all);
* BatchNorm stays un-synced (reference behaviour) with buffers broadcast from
  rank 0 like DataParallel's replica-0 semantics.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def enabled(self) -> bool:
        return self.world_size > 1


def env_info() -> DistInfo:
    return DistInfo(rank=int(os.environ.get("RANK", 0)),
                    world_size=int(os.environ.get("WORLD_SIZE", 1)),
                    local_rank=int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(backend: str | None = None, timeout_s: int = 600) -> DistInfo:
    """Initialise from torchrun-style env vars; no-op for a single process."""
    info = env_info()
    if info.world_size <= 1:
        return info
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    if use_gpu:
        torch.cuda.set_device(info.local_rank)
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=info.rank, world_size=info.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", info.local_rank)
        dist.init_process_group(**kw)
    info.backend = backend
    return info


def shutdown():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier():
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def wrap_ddp(model, device=None, bucket_cap_mb: float = 5.0, broadcast_buffers: bool = True,
             static_graph: bool = False):
    """DistributedDataParallel with RAFT-sized buckets (no-op single process)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    kw = dict(bucket_cap_mb=bucket_cap_mb, broadcast_buffers=broadcast_buffers,
              gradient_as_bucket_view=True, static_graph=static_graph)
    if device is not None and device.type == "cuda":
        kw["device_ids"] = [device.index]
        kw["output_device"] = device.index
    return DDP(model, **kw)


def unwrap(model):
    return model.module if hasattr(model, "module") else model


def all_reduce_mean(t: torch.Tensor) -> torch.Tensor:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t /= dist.get_world_size()
    return t


def all_reduce_max(x: float, device=None) -> float:
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([x], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())
    return x


def reduce_metrics(metrics: dict, device=None) -> dict:
    """Average a dict of scalars/0-d tensors over ranks with ONE all_reduce."""
    keys = sorted(metrics)
    if not keys:
        return {}
    vals = torch.stack([torch.as_tensor(metrics[k], dtype=torch.float64, device=device)
                        .reshape(()) for k in keys])
    vals = all_reduce_mean(vals)
    return {k: float(v) for k, v in zip(keys, vals.tolist())}
