#!/usr/bin/env python
"""Headline benchmark: RAFT (full, raft-things config) training throughput on
synthetic FlyingChairs-shaped pairs (368x496, 12 iterations, bf16, DDP over
RCCL), plus Sintel-resolution (1088x436, padded 1088x440) 12-iteration
inference FPS on rank 0.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1
the driver launches it under torch.distributed.run (one rank per GPU, RCCL).
Started directly with ``--gpus N>1`` (no WORLD_SIZE in the environment) it
re-launches itself the same way as a CHILD process before anything touches
the GPU and relays the child's exit code; rank 0's JSON line is the output.
W untimed steps, then exactly K timed steps bracketed by barrier +
synchronize; the MAX time over ranks is reported; rank 0 prints ONE JSON
line.  ``--device cpu`` runs the same step on CPU ranks over gloo (tests).

value = total image pairs / s over all N GPUs (weak scaling: fixed per-GPU
batch).  BASELINE.md publishes no training throughput (vs_baseline null for
the training value); the inference FPS is compared against the paper's
~10 fps (GTX 1080Ti, 1088x436) as ``inference.vs_baseline``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "train image-pairs/sec (node) + Sintel-res inference FPS, RAFT 12 iters"
BASELINE_INFER_FPS = 10.0  # RAFT paper, GTX 1080Ti, 1088x436


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="per-GPU batch (reference mixed schedule: 8)")
    ap.add_argument("--size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--iters", type=int, default=12)
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--fp32", action="store_true", help="disable bf16 autocast")
    ap.add_argument("--alternate-corr", action="store_true",
                    help="on-the-fly (memory-efficient) correlation instead of the all-pairs pyramid")
    ap.add_argument("--no-infer", action="store_true")
    ap.add_argument("--infer-size", type=int, nargs=2, default=[436, 1088])
    ap.add_argument("--infer-reps", type=int, default=20)
    ap.add_argument("--no-graph", action="store_true", help="eager inference instead of hipGraph")
    ap.add_argument("--train-graph", action="store_true",
                    help="one GPU: replay the whole training step (forward, loss, backward, clip, AdamW) "
                         "from one hipGraph (runtime/graph.py GraphedTrainStep).  Full RAFT: no faster than "
                         "the GPU-bound eager step, so off; RAFT-small (bf16, all-pairs, one GPU): on by "
                         "default -- its eager step is host-bound (host issue 11.5 ms = GPU 11.5 ms, "
                         "626-763 pairs/s run to run vs 748-750 replayed, profiles/r6/ab_small_graph_s32.txt)")
    ap.add_argument("--eager", action="store_true", help="force the eager training step")
    ap.add_argument("--corr-dtype", default="auto", choices=["auto", "float32", "bfloat16"],
                    help="all-pairs pyramid storage; auto = bf16 under bf16 autocast (EPE-drift gate: "
                         "tests/test_model_gpu.py::test_bf16_pyramid_epe_drift)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo ranks on the CPU (plumbing tests; reference-op path)")
    ap.add_argument("--reference-ops", action="store_true",
                    help="A/B baseline: run the model on stock PyTorch-ROCm ops only "
                         "(reference semantics: matmul volume, grid_sample lookup, unfused GRU)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def model_cfg_pyr(model) -> str:
    m = model.module if hasattr(model, "module") else model
    return "bf16" if str(m.cfg.pyr_dtype).endswith("bfloat16") else "fp32"


def launch_ranks(a) -> int:
    """``--gpus N`` without a launcher: run N ranks under torch.distributed.run
    as a child process (this process never initialises HIP) and relay its
    output and exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.parallel import dist as rdist
    from raft_stir_amd.train.loss import sequence_loss
    from raft_stir_amd.train.optim import fetch_optimizer
    from raft_stir_amd.data.synthetic import DevicePool

    if a.reference_ops:
        from raft_stir_amd.ops import _ext
        _ext.reference_mode().__enter__()
    cpu = a.device == "cpu"
    info = rdist.init_distributed(backend="gloo" if cpu else None)
    if info.world_size != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={info.world_size}")
    if cpu:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", info.local_rank)
        torch.cuda.set_device(dev)
    torch.manual_seed(1234)

    margs = make_args(small=a.small, mixed_precision=not a.fp32 and not cpu, corr_dtype=a.corr_dtype,
                      alternate_corr=a.alternate_corr)
    model = RAFT(margs).to(dev)
    if not cpu:
        model = model.to(memory_format=torch.channels_last)
    model.train()
    auto_graph = a.small and not a.fp32 and not a.alternate_corr and a.gpus == 1
    use_graph = (a.train_graph or auto_graph) and not a.eager and not cpu and not a.reference_ops
    if use_graph and info.world_size > 1:
        raise SystemExit("bench.py: --train-graph is one-GPU only (multi-GPU steps run eager under DDP)")
    targs = argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000)
    H, W = a.size
    pool = DevicePool(4, a.batch, H, W, dev, seed=info.rank * 97)

    if use_graph:
        # the same step, replayed from one hipGraph: the AdamW learning rate lives in
        # a device tensor that the (host-side) OneCycle scheduler updates between replays
        from raft_stir_amd.runtime.graph import GraphedTrainStep
        optimizer, scheduler = fetch_optimizer(targs, model, capturable=True)
        gstep = GraphedTrainStep(
            model, optimizer, lambda p, f, v: sequence_loss(p, f, v, gamma=0.8, sync_metrics=False)[0],
            pool.next(), clip=1.0, warmup=3, iters=a.iters)

        def step():
            loss = gstep.step(pool.next())
            scheduler.step()
            return loss
    else:
        ddp = rdist.wrap_ddp(model, device=dev)
        optimizer, scheduler = fetch_optimizer(targs, model)

        def step():
            i1, i2, flow, valid = pool.next()
            optimizer.zero_grad(set_to_none=True)
            preds = ddp(i1, i2, iters=a.iters)
            loss, _ = sequence_loss(preds, flow, valid, gamma=0.8, sync_metrics=False)
            loss.backward()
            if hasattr(optimizer, "clip_and_step"):  # clip + AdamW, two native launches
                optimizer.clip_and_step(1.0)
            else:
                torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
                optimizer.step()
            scheduler.step()
            return loss

    sync = (lambda: None) if cpu else torch.cuda.synchronize
    for _ in range(a.warmup):
        step()
    rdist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    sync()
    rdist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = rdist.all_reduce_max(elapsed, device=dev)
    ms = 1000.0 * elapsed / max(a.steps, 1)
    pairs_per_s = a.batch * info.world_size * a.steps / elapsed

    infer = None
    if info.is_main and not a.no_infer and not cpu:
        infer = bench_inference(model, dev, a)

    if info.is_main:
        out = {
            "metric": METRIC,
            "value": round(pairs_per_s, 3),
            "unit": "image-pairs/s",
            "n_gpus": info.world_size,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if (a.fp32 or cpu) else "bf16",
            "data": f"synthetic (FlyingChairs-shaped {H}x{W} pairs, random-init weights)",
            "config": {
                "model": "RAFT-small" if a.small else "RAFT (raft-things config, 5.26M params)",
                "global_batch": a.batch * info.world_size,
                "per_gpu_batch": a.batch,
                "seq_len": a.iters,
                "image_size": [H, W],
                "iters": a.iters,
                "parallelism": f"dp{info.world_size}",
                "ops": "stock-pytorch (reference semantics)" if (a.reference_ops or cpu) else "hip-kernels",
                "corr_pyramid": "fp32" if (a.reference_ops or cpu) else str(model_cfg_pyr(model)),
                "correlation": "on-the-fly" if a.alternate_corr else "all-pairs",
                "train_step": "hipgraph" if use_graph else "eager",
                "grad_allreduce": ("none" if info.world_size == 1 else
                                   "rccl: packed update-block buffer + DDP encoder buckets"
                                   if getattr(model.__dict__.get("_fused_train"), "grad_group", None)
                                   else f"{info.backend} DDP buckets"),
            },
            "final_loss": round(float(loss.detach()), 4),
            "inference": infer,
        }
        print(json.dumps(out), flush=True)
    rdist.shutdown()


@torch.no_grad()
def bench_inference(model, dev, a):
    from raft_stir_amd.utils.padder import InputPadder
    from raft_stir_amd.runtime.graph import GraphedInference
    net = model
    net.eval()
    h, w = a.infer_size
    g = torch.Generator(device=dev).manual_seed(0)
    i1 = torch.rand(1, 3, h, w, device=dev, generator=g) * 255
    i2 = torch.rand(1, 3, h, w, device=dev, generator=g) * 255
    padder = InputPadder(i1.shape)
    i1, i2 = padder.pad(i1, i2)
    if a.no_graph:
        run = lambda: net(i1, i2, iters=a.iters, test_mode=True)
        mode = "eager"
    else:
        gi = GraphedInference(net, i1.shape, iters=a.iters)
        run = lambda: gi(i1, i2)
        mode = "hipgraph"
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.infer_reps):
        run()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.infer_reps
    net.train()
    fps = 1.0 / dt
    return {"fps": round(fps, 2), "ms_per_pair": round(1000 * dt, 3), "batch": 1,
            "size": [h, w], "padded": list(i1.shape[-2:]), "iters": a.iters, "mode": mode,
            "vs_baseline": round(fps / BASELINE_INFER_FPS, 2)}


if __name__ == "__main__":
    main()
