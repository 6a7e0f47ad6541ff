"""Throughput of the real training feed: FlowDataset + FlowAugmentor + DataLoader.

The bench (bench.py) draws its batches from a device-resident synthetic pool,
so it never sees the host-side pipeline that ``train.py`` runs.  This script
measures that pipeline on its own: it writes synthetic FlyingChairs-format
files (512x384 ``.ppm`` pairs + ``.flo``, the release's layout) to a temporary
directory, builds the chairs stage exactly as ``train.py --stage chairs`` does
(``fetch_dataloader``: FlyingChairs + FlowAugmentor at the 368x496 crop, the
reference's augmentation parameters, /root/reference/core/datasets.py:199-234,
/root/reference/core/utils/augmentor.py:15-120) and times whole batches out of
the DataLoader with N worker processes.

    python scripts/bench_dataloader.py --workers 4 --batch 8 --batches 60
    python scripts/bench_dataloader.py --ranks 8 --workers 1   # 8 concurrent ranks (slowest rank reported)

Prints one JSON line: pairs/s per rank (one rank = one DataLoader), the
per-worker rate, and the engine's consumption rate it is compared against.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_chairs(root: str, n: int, h: int = 384, w: int = 512, seed: int = 0) -> None:
    from PIL import Image

    from raft_stir_amd.data import frame_utils
    rng = np.random.default_rng(seed)
    data = os.path.join(root, "FlyingChairs_release", "data")
    os.makedirs(data, exist_ok=True)
    ys, xs = np.mgrid[0:h, 0:w].astype(np.float32)
    for i in range(n):
        # smooth colour texture + an affine flow (values, not content, matter for timing)
        base = rng.random((h // 16 + 1, w // 16 + 1, 3)).astype(np.float32)
        img = np.asarray(Image.fromarray((base * 255).astype(np.uint8)).resize((w, h), Image.BICUBIC))
        a = rng.uniform(-0.05, 0.05, 4)
        t = rng.uniform(-20, 20, 2)
        flow = np.stack([t[0] + a[0] * (xs - w / 2) + a[1] * (ys - h / 2),
                         t[1] + a[2] * (xs - w / 2) + a[3] * (ys - h / 2)], -1).astype(np.float32)
        img2 = np.roll(img, (int(t[1]), int(t[0])), (0, 1))
        Image.fromarray(img).save(os.path.join(data, f"{i + 1:05d}_img1.ppm"))
        Image.fromarray(img2).save(os.path.join(data, f"{i + 1:05d}_img2.ppm"))
        frame_utils.writeFlow(os.path.join(data, f"{i + 1:05d}_flow.flo"), flow)
    np.savetxt(os.path.join(root, "FlyingChairs_release", "chairs_split.txt"), np.ones(n, dtype=np.int32), fmt="%d")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=8, help="per-rank batch (the bench's 8)")
    ap.add_argument("--batches", type=int, default=60, help="timed batches")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--files", type=int, default=256, help="synthetic pairs written")
    ap.add_argument("--engine-rate", type=float, default=386.0,
                    help="pairs/s per GPU the training engine consumes (round-3 headline)")
    ap.add_argument("--ranks", type=int, default=1,
                    help="concurrent ranks on this host (one DataLoader each, the data-parallel node's feed)")
    a = ap.parse_args()

    with tempfile.TemporaryDirectory() as root:
        t0 = time.perf_counter()
        write_chairs(root, a.files)
        t_write = time.perf_counter() - t0
        if a.ranks <= 1:
            rate = _measure(a, root, 0, None)
        else:
            import multiprocessing as mp
            ctx = mp.get_context("spawn")
            bar, q = ctx.Barrier(a.ranks), ctx.Queue()
            procs = [ctx.Process(target=_rank_main, args=(a, root, r, bar, q)) for r in range(a.ranks)]
            for p in procs:
                p.start()
            rates = [q.get(timeout=900) for _ in procs]
            for p in procs:
                p.join()
            rate = min(rates)
    print(json.dumps({
        "metric": "chairs training feed (FlowDataset + FlowAugmentor + DataLoader), pairs/s per rank",
        "pairs_per_s": round(rate, 1), "per_worker": round(rate / max(1, a.workers), 1),
        "workers": a.workers, "ranks": a.ranks, "batch": a.batch, "batches": a.batches, "crop": [368, 496],
        "engine_pairs_per_s": a.engine_rate, "feed_over_engine": round(rate / a.engine_rate, 2),
        "cpus_visible": os.cpu_count(), "cpus_usable": len(os.sched_getaffinity(0)), "write_s": round(t_write, 1),
    }))


def _rank_main(a, root, rank, bar, q):
    q.put(_measure(a, root, rank, bar))


def _measure(a, root, rank, bar):
    """pairs/s of one rank's DataLoader (the slowest rank bounds the step)."""
    import torch

    from raft_stir_amd.data.datasets import fetch_dataloader
    torch.set_num_threads(1)
    if True:
        args = argparse.Namespace(stage="chairs", image_size=[368, 496], batch_size=a.batch * a.ranks,
                                  num_workers=a.workers, data_root=root, seed=1234,
                                  chairs_split=os.path.join(root, "FlyingChairs_release", "chairs_split.txt"))
        loader = fetch_dataloader(args, rank=rank, world_size=a.ranks, pin_memory=False)
        it = iter(loader)
        n_done = 0

        def nxt():
            nonlocal it
            try:
                return next(it)
            except StopIteration:
                it = iter(loader)
                return next(it)
        for _ in range(a.warmup):
            nxt()
        if bar is not None:
            bar.wait()  # every rank's workers are up: time them concurrently
        t0 = time.perf_counter()
        for _ in range(a.batches):
            b = nxt()
            n_done += b[0].shape[0]
        dt = time.perf_counter() - t0
    return n_done / dt


if __name__ == "__main__":
    main()
