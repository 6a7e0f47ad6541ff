"""Optical-flow datasets and the per-stage training mixes
(reference core/datasets.py, same classes/constructor arguments/item contract).

Item contract (reference core/datasets.py:34-90):
  training:  (img1 (3,H,W) float [0,255], img2, flow (2,H,W) float, valid (H,W) float)
  test mode: (img1, img2, extra_info)
Dense datasets derive ``valid = |u| < 1000 & |v| < 1000``; sparse (KITTI/HD1K)
read it from the PNG.  Grayscale frames are tiled to 3 channels; RGBA is cut to RGB.

Engine additions:
  * every dataset takes ``root=`` (the reference hard-codes ``datasets/...``)
    and FlyingChairs takes ``split_file=`` (the reference reads
    ``chairs_split.txt`` from the CWD) -- defaults are unchanged;
  * ``FlyingChairs(split='train')`` is accepted as ``'training'`` (reference
    defect B10 made the default split empty);
  * ``fetch_dataloader`` adds the ``synthetic`` stage (FlyingChairs-shaped
    generated pairs, used by benchmarks/tests since no dataset ships offline),
    a rank-sharded resumable sampler (exact mid-epoch resume) and pinned
    memory for GPU training.
"""
from __future__ import annotations

import os
import os.path as osp
import random
from glob import glob

import numpy as np
import torch
import torch.utils.data as data

from . import frame_utils
from .augmentor import FlowAugmentor, SparseFlowAugmentor


class FlowDataset(data.Dataset):
    def __init__(self, aug_params=None, sparse=False):
        self.augmentor = None
        self.sparse = sparse
        if aug_params is not None:
            self.augmentor = (SparseFlowAugmentor if sparse else FlowAugmentor)(**aug_params)
        self.is_test = False
        self.init_seed = False
        self.flow_list = []
        self.image_list = []
        self.extra_info = []

    @staticmethod
    def _rgb(img):
        img = np.array(img).astype(np.uint8)
        if img.ndim == 2:
            return np.tile(img[..., None], (1, 1, 3))
        return img[..., :3]

    def _seed_worker(self):
        if self.init_seed:
            return
        info = torch.utils.data.get_worker_info()
        if info is not None:
            # reference seeds with the worker id; offset by the global rank so
            # data-parallel ranks draw different augmentations.
            rank = int(os.environ.get("RANK", 0))
            seed = info.id + 1000 * rank
            torch.manual_seed(seed)
            np.random.seed(seed)
            random.seed(seed)
            self.init_seed = True

    def __getitem__(self, index):
        if self.is_test:
            img1 = self._rgb(frame_utils.read_gen(self.image_list[index][0]))
            img2 = self._rgb(frame_utils.read_gen(self.image_list[index][1]))
            img1 = torch.from_numpy(img1).permute(2, 0, 1).float()
            img2 = torch.from_numpy(img2).permute(2, 0, 1).float()
            return img1, img2, self.extra_info[index]

        self._seed_worker()
        index = index % len(self.image_list)
        valid = None
        if self.sparse:
            flow, valid = frame_utils.readFlowKITTI(self.flow_list[index])
        else:
            flow = frame_utils.read_gen(self.flow_list[index])
        img1 = self._rgb(frame_utils.read_gen(self.image_list[index][0]))
        img2 = self._rgb(frame_utils.read_gen(self.image_list[index][1]))
        flow = np.array(flow).astype(np.float32)

        if self.augmentor is not None:
            if self.sparse:
                img1, img2, flow, valid = self.augmentor(img1, img2, flow, valid)
            else:
                img1, img2, flow = self.augmentor(img1, img2, flow)

        img1 = torch.from_numpy(np.ascontiguousarray(img1)).permute(2, 0, 1).float()
        img2 = torch.from_numpy(np.ascontiguousarray(img2)).permute(2, 0, 1).float()
        flow = torch.from_numpy(np.ascontiguousarray(flow)).permute(2, 0, 1).float()
        if valid is not None:
            valid = torch.from_numpy(np.ascontiguousarray(valid))
        else:
            valid = (flow[0].abs() < 1000) & (flow[1].abs() < 1000)
        return img1, img2, flow, valid.float()

    def __rmul__(self, v):
        self.flow_list = v * self.flow_list
        self.image_list = v * self.image_list
        return self

    def __len__(self):
        return len(self.image_list)


class MpiSintel(FlowDataset):
    def __init__(self, aug_params=None, split="training", root="datasets/Sintel", dstype="clean"):
        super().__init__(aug_params)
        flow_root = osp.join(root, split, "flow")
        image_root = osp.join(root, split, dstype)
        if split == "test":
            self.is_test = True
        scenes = sorted(os.listdir(image_root)) if osp.isdir(image_root) else []
        for scene in scenes:
            images = sorted(glob(osp.join(image_root, scene, "*.png")))
            for i in range(len(images) - 1):
                self.image_list.append([images[i], images[i + 1]])
                self.extra_info.append((scene, i))
            if split != "test":
                self.flow_list += sorted(glob(osp.join(flow_root, scene, "*.flo")))


_CHAIRS_INDEX = osp.join(osp.dirname(osp.abspath(__file__)), "chairs_val_index.txt")
_PACKAGED_SPLIT_NOTED = False


def load_chairs_split(split_file="chairs_split.txt", root=None) -> np.ndarray:
    """The FlyingChairs split (1 = training, 2 = validation per pair, reference
    chairs_split.txt; /root/reference/core/datasets.py:124-127).  A user file is
    looked up as given (CWD) and next to the data root; otherwise the packaged
    table (``chairs_val_index.txt``: the 640 validation indices of the
    22,872-pair release) is expanded."""
    cands = [split_file]
    if root is not None:
        cands.append(osp.join(root, "..", osp.basename(split_file)))
    for c in cands:
        if c and osp.exists(c):
            return np.loadtxt(c, dtype=np.int32).reshape(-1)
    global _PACKAGED_SPLIT_NOTED
    if not _PACKAGED_SPLIT_NOTED:
        _PACKAGED_SPLIT_NOTED = True
        print(f"FlyingChairs: {split_file} not found; using the packaged 22,872-pair split table", flush=True)
    total, idx = None, []
    with open(_CHAIRS_INDEX) as f:
        for line in f:
            if line.startswith("#"):
                if line.startswith("# total"):
                    total = int(line.split()[2])
                continue
            idx.extend(int(v) for v in line.split())
    out = np.ones(total, dtype=np.int32)
    out[np.asarray(idx, dtype=np.int64)] = 2
    return out


class FlyingChairs(FlowDataset):
    def __init__(self, aug_params=None, split="train", root="datasets/FlyingChairs_release/data",
                 split_file="chairs_split.txt"):
        super().__init__(aug_params)
        split = {"train": "training", "val": "validation"}.get(split, split)
        images = sorted(glob(osp.join(root, "*.ppm")))
        flows = sorted(glob(osp.join(root, "*.flo")))
        assert len(images) // 2 == len(flows)
        if not flows:
            return
        split_list = load_chairs_split(split_file, root)
        # a split table for a different release would silently mislabel pairs
        if len(split_list) != len(flows):
            raise ValueError(
                f"FlyingChairs: split file {split_file!r} has {len(split_list)} entries but {root!r} holds "
                f"{len(flows)} flow files; pass split_file= a table with one line (1 = train, 2 = val) per "
                f"flow file of this directory (the packaged table is for the full 22,872-pair release)")
        want = {"training": 1, "validation": 2}.get(split)
        for i in range(len(flows)):
            if split_list[i] == want:
                self.flow_list.append(flows[i])
                self.image_list.append([images[2 * i], images[2 * i + 1]])


class FlyingThings3D(FlowDataset):
    def __init__(self, aug_params=None, root="datasets/FlyingThings3D", dstype="frames_cleanpass"):
        super().__init__(aug_params)
        for cam in ["left"]:
            for direction in ["into_future", "into_past"]:
                image_dirs = sorted(osp.join(f, cam) for f in glob(osp.join(root, dstype, "TRAIN/*/*")))
                flow_dirs = sorted(osp.join(f, direction, cam)
                                   for f in glob(osp.join(root, "optical_flow/TRAIN/*/*")))
                for idir, fdir in zip(image_dirs, flow_dirs):
                    images = sorted(glob(osp.join(idir, "*.png")))
                    flows = sorted(glob(osp.join(fdir, "*.pfm")))
                    for i in range(len(flows) - 1):
                        if direction == "into_future":
                            self.image_list.append([images[i], images[i + 1]])
                            self.flow_list.append(flows[i])
                        else:
                            self.image_list.append([images[i + 1], images[i]])
                            self.flow_list.append(flows[i + 1])


class KITTI(FlowDataset):
    def __init__(self, aug_params=None, split="training", root="datasets/KITTI"):
        super().__init__(aug_params, sparse=True)
        if split == "testing":
            self.is_test = True
        root = osp.join(root, split)
        images1 = sorted(glob(osp.join(root, "image_2/*_10.png")))
        images2 = sorted(glob(osp.join(root, "image_2/*_11.png")))
        for img1, img2 in zip(images1, images2):
            self.extra_info.append([osp.basename(img1)])
            self.image_list.append([img1, img2])
        if split == "training":
            self.flow_list = sorted(glob(osp.join(root, "flow_occ/*_10.png")))


class HD1K(FlowDataset):
    def __init__(self, aug_params=None, root="datasets/HD1k"):
        super().__init__(aug_params, sparse=True)
        seq = 0
        while True:
            flows = sorted(glob(osp.join(root, "hd1k_flow_gt", "flow_occ/%06d_*.png" % seq)))
            images = sorted(glob(osp.join(root, "hd1k_input", "image_2/%06d_*.png" % seq)))
            if not flows:
                break
            for i in range(len(flows) - 1):
                self.flow_list.append(flows[i])
                self.image_list.append([images[i], images[i + 1]])
            seq += 1


class SyntheticChairs(data.Dataset):
    """Generated FlyingChairs-shaped pairs with the FlowDataset contract."""

    def __init__(self, length=22232, size=(368, 496), seed=0, sparse=False):
        from .synthetic import SyntheticFlowDataset
        self.inner = SyntheticFlowDataset(length, size, seed, sparse)

    def __len__(self):
        return len(self.inner)

    def __getitem__(self, i):
        return self.inner[i]


def _root(args, name, default):
    base = getattr(args, "data_root", None)
    return osp.join(base, name) if base else default


def build_train_dataset(args, TRAIN_DS="C+T+K+S+H"):
    size = list(args.image_size)
    if args.stage == "synthetic":
        return SyntheticChairs(length=getattr(args, "synthetic_length", 22232), size=size)
    if args.stage == "chairs":
        aug = {"crop_size": size, "min_scale": -0.1, "max_scale": 1.0, "do_flip": True}
        return FlyingChairs(aug, split="training",
                            root=_root(args, "FlyingChairs_release/data",
                                       "datasets/FlyingChairs_release/data"),
                            split_file=getattr(args, "chairs_split", "chairs_split.txt"))
    things_root = _root(args, "FlyingThings3D", "datasets/FlyingThings3D")
    if args.stage == "things":
        aug = {"crop_size": size, "min_scale": -0.4, "max_scale": 0.8, "do_flip": True}
        clean = FlyingThings3D(aug, root=things_root, dstype="frames_cleanpass")
        final = FlyingThings3D(aug, root=things_root, dstype="frames_finalpass")
        return clean + final
    if args.stage == "sintel":
        aug = {"crop_size": size, "min_scale": -0.2, "max_scale": 0.6, "do_flip": True}
        sintel_root = _root(args, "Sintel", "datasets/Sintel")
        things = FlyingThings3D(aug, root=things_root, dstype="frames_cleanpass")
        clean = MpiSintel(aug, split="training", root=sintel_root, dstype="clean")
        final = MpiSintel(aug, split="training", root=sintel_root, dstype="final")
        if TRAIN_DS == "C+T+K+S+H":
            kitti = KITTI({"crop_size": size, "min_scale": -0.3, "max_scale": 0.5, "do_flip": True},
                          root=_root(args, "KITTI", "datasets/KITTI"))
            hd1k = HD1K({"crop_size": size, "min_scale": -0.5, "max_scale": 0.2, "do_flip": True},
                        root=_root(args, "HD1k", "datasets/HD1k"))
            return 100 * clean + 100 * final + 200 * kitti + 5 * hd1k + things
        if TRAIN_DS == "C+T+K/S":
            return 100 * clean + 100 * final + things
        raise ValueError(f"unknown TRAIN_DS {TRAIN_DS!r}")
    if args.stage == "kitti":
        aug = {"crop_size": size, "min_scale": -0.2, "max_scale": 0.4, "do_flip": False}
        return KITTI(aug, split="training", root=_root(args, "KITTI", "datasets/KITTI"))
    raise ValueError(f"unknown stage {args.stage!r}")


class ResumableSampler(data.Sampler):
    """Shuffled, rank-sharded, *resumable* sampler.

    The permutation of epoch ``e`` is drawn from ``Generator(seed + e)``, so it
    is identical on every rank and after a restart; rank ``r`` takes every
    ``world_size``-th index (drop_last semantics), and :meth:`set_position`
    skips the batches already consumed in the current epoch -- a resumed run
    sees exactly the samples the uninterrupted run would have.
    """

    def __init__(self, dataset, rank=0, world_size=1, seed=0, batch_size=1):
        self.n = len(dataset)
        self.rank, self.world_size, self.seed = rank, world_size, seed
        self.batch_size = batch_size
        self.per_rank = self.n // world_size
        self.epoch = 0
        self.skip = 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def set_position(self, epoch, batches_done):
        self.epoch, self.skip = epoch, batches_done * self.batch_size

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        perm = torch.randperm(self.n, generator=g)[: self.per_rank * self.world_size]
        mine = perm[self.rank::self.world_size].tolist()
        skip, self.skip = self.skip, 0
        return iter(mine[skip:])

    def __len__(self):
        return self.per_rank


# Chairs feed on MI355X boxes (scripts/bench_dataloader.py, profiles/r5/feed_s29.jsonl):
# ~50-70 pairs/s per worker; the engine consumes ~427 pairs/s per GPU, so 12
# workers per rank (600 pairs/s, 1.4x the engine) when the CPUs allow it.
FEED_WORKERS = 12


def auto_workers(local_ranks=None) -> int:
    """DataLoader workers per rank: FEED_WORKERS, capped by this process's CPU
    share (CPUs in its affinity mask / ranks on the node, one kept for the
    training process itself)."""
    if local_ranks is None:
        local_ranks = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:
        cpus = os.cpu_count() or 1
    return max(0, min(FEED_WORKERS, cpus // max(1, local_ranks) - 1))


def fetch_dataloader(args, TRAIN_DS="C+T+K+S+H", rank=None, world_size=None, pin_memory=None):
    """Per-stage DataLoader (reference core/datasets.py:199-234).

    ``args.batch_size`` is the GLOBAL batch like the reference; under
    torch.distributed each rank loads ``batch_size // world_size`` samples
    through a DistributedSampler."""
    train_dataset = build_train_dataset(args, TRAIN_DS)
    if world_size is None:
        world_size = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if rank is None:
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
    per_rank = max(1, args.batch_size // world_size)
    sampler = ResumableSampler(train_dataset, rank=rank, world_size=world_size,
                               seed=int(getattr(args, "seed", 1234)), batch_size=per_rank)
    workers = getattr(args, "num_workers", None)
    workers = auto_workers() if workers is None or int(workers) < 0 else int(workers)
    if pin_memory is None:
        pin_memory = torch.cuda.is_available()
    loader = data.DataLoader(train_dataset, batch_size=per_rank, pin_memory=pin_memory,
                             sampler=sampler, num_workers=workers, drop_last=True,
                             persistent_workers=False)
    if rank == 0:
        print("Training with %d image pairs" % len(train_dataset))
    return loader
