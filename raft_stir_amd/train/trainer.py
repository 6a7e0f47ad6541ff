"""Supervised RAFT training (reference train.py:136-247), one process per GPU.

CLI-compatible with the reference (same flags and defaults: --name --stage
--restore_ckpt --small --validation --lr --num_steps --batch_size
--image_size --gpus --mixed_precision --iters --wdecay --epsilon --clip
--dropout --gamma --add_noise) plus engine flags (see :func:`build_parser`).

Per step (reference train.py:162-183):
    zero_grad -> H2D (pinned, non_blocking) -> optional Gaussian noise
    (sigma ~ U(0,5), now drawn on the device per rank) -> forward (12 iters)
    -> sequence_loss -> backward (DDP all-reduces gradient buckets over
    RCCL while the backward is still running) -> clip_grad_norm(clip) ->
    AdamW step -> OneCycle step -> log.

Engine differences:
  * ``nn.DataParallel`` (broadcast + gather to GPU0 every step) is replaced by
    DistributedDataParallel, one process per GPU: launched by torchrun, or
    spawned here when ``--gpus`` lists several devices without torchrun;
    ``--batch_size`` stays the GLOBAL batch (split evenly across ranks);
  * ``--mixed_precision`` means bf16 autocast (bf16 has fp32's exponent range,
    so no loss scaling; the GradScaler is kept, disabled, for API parity);
  * non-finite gradients are detected on the device and the optimizer step is
    skipped without a host sync (fused AdamW ``found_inf``), with a skip
    counter logged and an abort after ``--max_skips`` consecutive skips;
  * every ``--val_freq`` steps the reference-layout weights
    ``checkpoints/<step>_<name>.pth`` AND a full resume point
    ``checkpoints/<name>_resume_<step>.pt`` are written (rank 0, atomically);
    ``--resume auto`` continues from the newest one (model, optimizer,
    schedule, step, RNG);
  * ``--fault_at_step K`` raises at step K (fault-injection for resume tests).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

from ..config import make_args
from ..models import RAFT
from ..parallel import dist as rdist
from . import checkpoint as ckpt
from .logger import Logger
from .loss import sequence_loss
from .optim import count_parameters, fetch_optimizer


def build_parser():
    p = argparse.ArgumentParser(description="RAFT training (MI355X engine)")
    p.add_argument("--name", default="raft", help="name your experiment")
    p.add_argument("--stage", help="chairs | things | sintel | kitti | synthetic")
    p.add_argument("--restore_ckpt", help="restore checkpoint (weights only, strict=False)")
    p.add_argument("--small", action="store_true", help="use small model")
    p.add_argument("--validation", type=str, nargs="+", default=[])
    p.add_argument("--lr", type=float, default=0.00002)
    p.add_argument("--num_steps", type=int, default=100000)
    p.add_argument("--batch_size", type=int, default=6, help="global batch (all ranks)")
    p.add_argument("--image_size", type=int, nargs="+", default=[384, 512])
    p.add_argument("--gpus", type=int, nargs="+", default=[0, 1])
    p.add_argument("--mixed_precision", action="store_true", help="bf16 autocast")
    p.add_argument("--iters", type=int, default=12)
    p.add_argument("--wdecay", type=float, default=0.00005)
    p.add_argument("--epsilon", type=float, default=1e-8)
    p.add_argument("--clip", type=float, default=1.0)
    p.add_argument("--dropout", type=float, default=0.0)
    p.add_argument("--gamma", type=float, default=0.8, help="exponential weighting")
    p.add_argument("--add_noise", action="store_true")
    # engine flags
    p.add_argument("--alternate_corr", action="store_true",
                   help="on-the-fly (memory-efficient) correlation, differentiable")
    p.add_argument("--data_root", default=None, help="parent of FlyingChairs_release/, Sintel/, ...")
    p.add_argument("--chairs_split", default="chairs_split.txt")
    p.add_argument("--num_workers", type=int, default=None,
                   help="DataLoader workers per rank (default: data.datasets.auto_workers, up to 12)")
    p.add_argument("--ckpt_dir", default="checkpoints")
    p.add_argument("--log_dir", default=None, help="JSONL/TensorBoard dir (default runs/<name>)")
    p.add_argument("--val_freq", type=int, default=5000)
    p.add_argument("--sum_freq", type=int, default=100)
    p.add_argument("--resume", default=None, help="'auto' or a *_resume_*.pt path")
    p.add_argument("--max_skips", type=int, default=100,
                   help="abort after this many consecutive non-finite steps")
    p.add_argument("--fault_at_step", type=int, default=-1, help="fault injection (tests)")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--device", default=None, help="force cpu / cuda")
    p.add_argument("--synthetic_length", type=int, default=22232)
    p.add_argument("--bucket_mb", type=float, default=5.0, help="DDP gradient bucket size")
    p.add_argument("--deterministic", action="store_true",
                   help="bitwise-reproducible GPU steps: ordered reductions instead of fp32 atomics, "
                        "fixed-point on-the-fly correlation backward (runtime/determinism.py)")
    return p


class NonFiniteError(RuntimeError):
    pass


class InjectedFault(RuntimeError):
    pass


def _device(args, info):
    if args.device:
        return torch.device(args.device if args.device != "cuda" else f"cuda:{info.local_rank}")
    if torch.cuda.is_available():
        return torch.device("cuda", info.local_rank)
    return torch.device("cpu")


def train(args):
    info = rdist.init_distributed(backend="gloo" if args.device == "cpu" else None)
    dev = _device(args, info)
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    torch.manual_seed(args.seed + info.rank)
    np.random.seed(args.seed + info.rank)

    if getattr(args, "deterministic", False):
        from ..runtime.determinism import set_deterministic
        set_deterministic(True)
    margs = make_args(small=args.small, mixed_precision=args.mixed_precision,
                      alternate_corr=args.alternate_corr, dropout=args.dropout,
                      deterministic=getattr(args, "deterministic", False))
    model = RAFT(margs)
    if info.is_main:
        print("Parameter Count: %d" % count_parameters(model))
    if args.restore_ckpt is not None:
        ckpt.load_weights(model, args.restore_ckpt, strict=False)
    model.to(dev)
    if dev.type == "cuda":
        model.to(memory_format=torch.channels_last)
    model.train()
    if args.stage != "chairs":
        model.freeze_bn()

    from ..data.datasets import fetch_dataloader
    train_loader = fetch_dataloader(args, rank=info.rank, world_size=info.world_size)
    optimizer, scheduler = fetch_optimizer(args, model)
    scaler = torch.amp.GradScaler("cuda", enabled=False)  # bf16 needs no loss scaling

    noise_gen = None
    if args.add_noise:
        noise_gen = torch.Generator(device=dev)
        noise_gen.manual_seed(args.seed * 7919 + info.rank)
    generators = {"noise": noise_gen} if noise_gen is not None else {}
    start_step, start_epoch, start_batch = 0, 0, 0
    resume_path = ckpt.latest_resume(args.ckpt_dir, args.name) if args.resume == "auto" else args.resume
    if resume_path:
        obj = ckpt.load_resume(resume_path, model, optimizer, scheduler, scaler,
                               map_location="cpu", restore_rng=True)
        start_step = int(obj["step"])
        start_epoch = int(obj["extra"].get("epoch", 0))
        start_batch = int(obj["extra"].get("batch", 0))
        # each rank's own RNG streams (+ the noise generator) from its sidecar
        ckpt.load_rank_rng(resume_path, info.rank, generators)
        if info.is_main:
            print(f"resumed from {resume_path} at step {start_step}")

    ddp = rdist.wrap_ddp(model, device=dev, bucket_cap_mb=args.bucket_mb)
    log_dir = args.log_dir or os.path.join("runs", args.name)
    per_rank = max(1, args.batch_size // info.world_size)
    logger = Logger(model, scheduler, sum_freq=args.sum_freq, log_dir=log_dir, rank=info.rank,
                    pairs_per_step=per_rank * info.world_size, reduce_fn=rdist.all_reduce_mean,
                    start_step=start_step)

    fused_opt = any(g.get("fused") for g in optimizer.param_groups)
    params = [p for p in model.parameters() if p.requires_grad]
    skipped = torch.zeros((), device=dev)
    consecutive = torch.zeros((), device=dev)
    if info.is_main:
        os.makedirs(args.ckpt_dir, exist_ok=True)

    total_steps = start_step
    epoch, batch_in_epoch = start_epoch, start_batch
    sampler = getattr(train_loader, "sampler", None)
    should_keep_training = total_steps <= args.num_steps
    while should_keep_training:
        if hasattr(sampler, "set_position"):
            sampler.set_position(epoch, batch_in_epoch)  # exact mid-epoch resume
        elif hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        for data_blob in train_loader:
            batch_in_epoch += 1
            if total_steps == args.fault_at_step:
                raise InjectedFault(f"injected fault at step {total_steps}")
            optimizer.zero_grad(set_to_none=True)
            image1, image2, flow, valid = [x.to(dev, non_blocking=True) for x in data_blob]
            if noise_gen is not None:
                stdv = torch.rand((), device=dev, generator=noise_gen) * 5.0
                image1 = (image1 + stdv * torch.randn(image1.shape, device=dev, generator=noise_gen)
                          ).clamp(0.0, 255.0)
                image2 = (image2 + stdv * torch.randn(image2.shape, device=dev, generator=noise_gen)
                          ).clamp(0.0, 255.0)

            flow_predictions = ddp(image1, image2, iters=args.iters)
            loss, metrics = sequence_loss(flow_predictions, flow, valid, args.gamma,
                                          sync_metrics=False)
            loss.backward()
            if hasattr(optimizer, "clip_and_step"):
                # clip + AdamW in two native launches; a non-finite norm skips
                # the update on the device (train/optim.py FusedClipAdamW)
                total_norm = optimizer.clip_and_step(args.clip)
                found_inf = (~torch.isfinite(total_norm)).float()
            else:
                total_norm = torch.nn.utils.clip_grad_norm_(params, args.clip)
                found_inf = (~torch.isfinite(total_norm)).float()
                if fused_opt:
                    optimizer.found_inf = found_inf   # fused AdamW skips the update on the device
                    optimizer.step()
                elif float(found_inf) == 0.0:
                    optimizer.step()
            scheduler.step()
            skipped += found_inf
            consecutive = (consecutive + found_inf) * found_inf
            metrics["skipped"] = skipped
            logger.push(metrics)
            if (total_steps + 1) % args.sum_freq == 0 and float(consecutive) >= args.max_skips:
                raise NonFiniteError(f"{int(consecutive)} consecutive non-finite steps")

            if total_steps % args.val_freq == args.val_freq - 1:
                resume_file = os.path.join(args.ckpt_dir, "%s_resume_%d.pt" % (args.name, total_steps + 1))
                ckpt.save_rank_rng(resume_file, info.rank, generators)
                if info.is_main:
                    ckpt.save_weights(model, os.path.join(args.ckpt_dir, "%d_%s.pth" % (total_steps + 1, args.name)))
                    ckpt.save_resume(resume_file, model, optimizer, scheduler, scaler, step=total_steps + 1,
                                     extra={"epoch": epoch, "batch": batch_in_epoch})
                    results = run_validation(model, args)
                    logger.write_dict(results)
                rdist.barrier()
                model.train()
                if args.stage != "chairs":
                    model.freeze_bn()

            total_steps += 1
            if total_steps > args.num_steps:
                should_keep_training = False
                break
        else:
            epoch, batch_in_epoch = epoch + 1, 0

    logger.close()
    path = os.path.join(args.ckpt_dir, "%s.pth" % args.name)
    if info.is_main:
        ckpt.save_weights(model, path)
    rdist.barrier()
    return path


def run_validation(model, args):
    from ..eval import evaluate
    results = {}
    for name in args.validation or []:
        fn = evaluate.VALIDATORS.get(name)
        if fn is None:
            continue
        kw = {}
        if args.data_root:
            sub = {"chairs": "FlyingChairs_release/data", "sintel": "Sintel", "kitti": "KITTI"}[name]
            kw["root"] = os.path.join(args.data_root, sub)
        try:
            results.update(fn(model, **kw))
        except (FileNotFoundError, AssertionError, OSError) as e:
            print(f"validation {name} skipped: {e}")
    return results


def _spawn_worker(local_rank, gpus, argv, port):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(len(gpus)),
                      LOCAL_WORLD_SIZE=str(len(gpus)), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ["HIP_VISIBLE_DEVICES"] = ",".join(str(g) for g in gpus)
    args = build_parser().parse_args(argv)
    train(args)
    rdist.shutdown()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = build_parser().parse_args(argv)
    np.random.seed(args.seed)
    torch.manual_seed(args.seed)
    launched = "WORLD_SIZE" in os.environ
    ngpu = torch.cuda.device_count()  # does not initialise HIP
    # RS_SPAWN_CPU=1: the same spawn path with CPU (gloo) ranks (tests/test_distributed_cpu.py)
    cpu_spawn = os.environ.get("RS_SPAWN_CPU") == "1" and args.device == "cpu"
    if not launched and len(args.gpus) > 1 and ((ngpu > 1 and args.device != "cpu") or cpu_spawn):
        # the reference's `--gpus 0 1` -> one process per GPU (DDP over RCCL)
        import torch.multiprocessing as mp
        port = 29500 + (os.getpid() % 1000)
        mp.start_processes(_spawn_worker, args=(args.gpus, argv, port), nprocs=len(args.gpus),
                           start_method="spawn")
        return os.path.join(args.ckpt_dir, "%s.pth" % args.name)
    path = train(args)
    rdist.shutdown()
    return path
