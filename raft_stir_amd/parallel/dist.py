"""Process-group setup and data parallelism over RCCL (xGMI) / gloo.

Replaces the reference's single-process ``nn.DataParallel`` (train.py:138;
broadcast of all parameters every forward, gather of 12 full-resolution
predictions to GPU0, reduce of gradients to GPU0 -- SURVEY §2.5) with one
process per GPU:

* ``torch.distributed`` backend ``nccl`` (= RCCL on ROCm) for GPUs, ``gloo``
  for CPU ranks (tests);
* gradients all-reduced *during* backward, in two parts:
  - the update block (~57 % of RAFT's 21 MB of fp32 gradients) is trained by
    the fused engine (models/fused_train.py), whose weight gradients land in
    ONE packed fp32 buffer on the weight-gradient HIP stream.  That buffer is
    all-reduced as a single RCCL collective issued from that stream the
    moment the last iteration-batched wgrad GEMM is queued -- i.e. while the
    encoder backward is still running on the main stream -- and DDP is told
    to ignore those parameters;
  - the encoder gradients go through DDP's reducer buckets (hooks on
    AccumulateGrad, ~5 MB buckets, RCCL stream), which fire as the encoder
    backward produces them.
  On an 8 x MI355X node a ring over the 7 xGMI links moves ~37 MB per rank
  per step -- a fraction of a millisecond -- and nothing of it sits at the
  end of backward except the last encoder bucket.
  Stream budget per process (GPU_MAX_HW_QUEUES = 4): main, side 0 (context
  encoder / flow branch / pyramid-gradient scatter), side 1 (weight
  gradients + the packed all-reduce issue point), and the process group's
  RCCL stream;
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


def init_distributed(backend: str | None = None, timeout_s: int = 600, force: bool = False) -> DistInfo:
    """Initialise from torchrun-style env vars; no-op for a single process
    unless ``force`` (a world of one, e.g. to exercise RCCL on one GPU)."""
    info = env_info()
    if info.world_size <= 1 and not force:
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
             static_graph: bool = False, force: bool = False, packed_update_grads: bool | None = None):
    """DistributedDataParallel with RAFT-sized buckets.

    No-op for a single process unless ``force`` (wraps a world of one, so the
    DDP/RCCL path can be exercised on one GPU).  ``packed_update_grads``
    (default: whenever the fused training engine will train the update
    block) hands the update-block gradients to the engine's packed
    all-reduce and makes DDP ignore those parameters (module docstring)."""
    if not (dist.is_available() and dist.is_initialized()):
        return model
    if dist.get_world_size() == 1 and not force:
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    if packed_update_grads is None:
        packed_update_grads = _fused_train_capable(model, device)
    if packed_update_grads:
        eng = model._train_engine()
        ids = {id(p) for p in eng.params}
        names = [n for n, p in model.named_parameters() if id(p) in ids]
        # DDP does not broadcast ignored parameters: replicate them from rank 0 here
        with torch.no_grad():
            for p in eng.params:
                dist.broadcast(p.data, 0)
        DDP._set_params_and_buffers_to_ignore_for_model(model, names)
        eng.attach_grad_group(dist.group.WORLD, dist.get_world_size())
    kw = dict(bucket_cap_mb=bucket_cap_mb, broadcast_buffers=broadcast_buffers,
              gradient_as_bucket_view=True, static_graph=static_graph)
    if device is not None and device.type == "cuda":
        kw["device_ids"] = [device.index]
        kw["output_device"] = device.index
    return DDP(model, **kw)


def _fused_train_capable(model, device) -> bool:
    """Will RAFT training on ``device`` run through the fused training engine?"""
    cfg = getattr(model, "cfg", None)
    if cfg is None or not hasattr(model, "_train_engine") or device is None or device.type != "cuda":
        return False
    from ..models.fused_train import FusedTrainEngine
    return FusedTrainEngine.config_capable(cfg)


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
