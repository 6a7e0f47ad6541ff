"""Checkpoints: reference-compatible weights + full training resume.

Reference behaviour (reference train.py:141-142, 185-187, 211-212):
  * ``torch.save(model.state_dict())`` of the ``nn.DataParallel`` wrapper, so
    every key carries a ``module.`` prefix; tools load by wrapping in
    DataParallel first;
  * restore is ``load_state_dict(torch.load(path), strict=False)`` -- weights
    only, a stage-to-stage warm start.

Here:
  * :func:`load_weights` accepts files with or without ``module.`` (and
    DDP / torch.compile ``_orig_mod.`` prefixes), always via
    ``torch.load(weights_only=True)``; it reports missing/unexpected keys;
  * :func:`save_weights` writes the reference layout (fp32 tensors, the
    reference key names, ``module.`` prefix by default) so reference tools and
    STIRMetrics load our checkpoints unchanged;
  * :func:`save_resume` / :func:`load_resume` add what the reference lacks: a
    full resume point (model, optimizer, LR schedule, grad scaler, step,
    CPU/CUDA/numpy/python RNG states), written atomically (tmp + rename) so a
    crash mid-write never corrupts the latest checkpoint;
  * :func:`latest_resume` finds the newest resume file in a directory.
"""
from __future__ import annotations

import glob
import os
import random
import re
from typing import Dict, Optional

import numpy as np
import torch

_PREFIXES = ("module.", "_orig_mod.")


def strip_prefix(state: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    out = {}
    for k, v in state.items():
        changed = True
        while changed:
            changed = False
            for p in _PREFIXES:
                if k.startswith(p):
                    k = k[len(p):]
                    changed = True
        out[k] = v
    return out


def _unwrap(model):
    while hasattr(model, "module"):
        model = model.module
    return getattr(model, "_orig_mod", model)


def load_weights(model, path_or_state, strict: bool = False, map_location="cpu", verbose=True):
    """Load reference-layout weights into ``model`` (DP/DDP-wrapped or not)."""
    if isinstance(path_or_state, (str, os.PathLike)):
        state = torch.load(path_or_state, map_location=map_location, weights_only=True)
    else:
        state = path_or_state
    if isinstance(state, dict) and "model" in state and isinstance(state["model"], dict):
        state = state["model"]  # a resume file
    state = strip_prefix(state)
    res = _unwrap(model).load_state_dict(state, strict=strict)
    if verbose and (res.missing_keys or res.unexpected_keys):
        print(f"load_weights: missing={len(res.missing_keys)} unexpected={len(res.unexpected_keys)}")
    return res


def reference_state_dict(model, prefix: str = "module.") -> Dict[str, torch.Tensor]:
    """fp32, CPU, reference key names (optionally DataParallel-prefixed)."""
    sd = _unwrap(model).state_dict()
    out = {}
    for k, v in sd.items():
        t = v.detach().cpu()
        if t.is_floating_point():
            t = t.float().contiguous()
        out[prefix + k] = t
    return out


def _atomic_save(obj, path: str):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_weights(model, path: str, dp_prefix: bool = True):
    _atomic_save(reference_state_dict(model, "module." if dp_prefix else ""), path)


def _rng_state():
    st = {"torch": torch.get_rng_state(), "numpy": np.random.get_state(),
          "python": random.getstate()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def _set_rng_state(st):
    if not st:
        return
    torch.set_rng_state(st["torch"])
    np.random.set_state(st["numpy"])
    random.setstate(st["python"])
    if "cuda" in st and torch.cuda.is_available():
        try:
            torch.cuda.set_rng_state_all(st["cuda"])
        except Exception:
            pass


def _np_state_to_safe(st):
    # numpy's legacy state tuple -> plain lists/tensors so weights_only loads it
    name, keys, pos, has_gauss, cached = st
    return {"name": name, "keys": torch.from_numpy(np.asarray(keys, np.int64)), "pos": int(pos),
            "has_gauss": int(has_gauss), "cached": float(cached)}


def _np_state_from_safe(d):
    return (d["name"], d["keys"].numpy().astype(np.uint32), d["pos"], d["has_gauss"], d["cached"])


def save_resume(path: str, model, optimizer=None, scheduler=None, scaler=None, step: int = 0,
                extra: Optional[dict] = None):
    rng = _rng_state()
    rng["numpy"] = _np_state_to_safe(rng["numpy"])
    py = rng["python"]
    rng["python"] = [py[0], list(py[1]), py[2]]
    obj = {
        "format": "raft_stir_amd.resume/1",
        "model": reference_state_dict(model, prefix=""),
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "scheduler": scheduler.state_dict() if scheduler is not None else None,
        "scaler": scaler.state_dict() if scaler is not None else None,
        "step": int(step),
        "rng": rng,
        "extra": extra or {},
    }
    _atomic_save(obj, path)


def load_resume(path: str, model, optimizer=None, scheduler=None, scaler=None,
                map_location="cpu", restore_rng: bool = True) -> dict:
    obj = torch.load(path, map_location=map_location, weights_only=True)
    assert obj.get("format", "").startswith("raft_stir_amd.resume"), f"{path}: not a resume file"
    _unwrap(model).load_state_dict(obj["model"], strict=True)
    if optimizer is not None and obj.get("optimizer"):
        optimizer.load_state_dict(obj["optimizer"])
    if scheduler is not None and obj.get("scheduler"):
        scheduler.load_state_dict(obj["scheduler"])
    if scaler is not None and obj.get("scaler"):
        scaler.load_state_dict(obj["scaler"])
    if restore_rng and obj.get("rng"):
        rng = dict(obj["rng"])
        rng["numpy"] = _np_state_from_safe(rng["numpy"])
        py = rng["python"]
        rng["python"] = (py[0], tuple(py[1]), py[2])
        _set_rng_state(rng)
    return obj


def rank_rng_path(path: str, rank: int) -> str:
    return f"{path}.rank{rank}.rng"


def save_rank_rng(path: str, rank: int, generators: Optional[dict] = None):
    """Per-rank RNG sidecar of a resume file: every rank's own CPU/CUDA/numpy/
    python RNG streams plus named extra generators (e.g. the --add_noise
    generator), so a resumed multi-rank run continues each rank's streams
    instead of giving every rank rank 0's."""
    rng = _rng_state()
    rng["numpy"] = _np_state_to_safe(rng["numpy"])
    py = rng["python"]
    rng["python"] = [py[0], list(py[1]), py[2]]
    rng["generators"] = {k: g.get_state() for k, g in (generators or {}).items()}
    _atomic_save({"format": "raft_stir_amd.rank_rng/1", "rank": int(rank), "rng": rng}, rank_rng_path(path, rank))


def load_rank_rng(path: str, rank: int, generators: Optional[dict] = None) -> bool:
    """Restore this rank's sidecar (written by save_rank_rng); False if absent."""
    side = rank_rng_path(path, rank)
    if not os.path.exists(side):
        return False
    obj = torch.load(side, map_location="cpu", weights_only=True)
    assert obj.get("format", "").startswith("raft_stir_amd.rank_rng") and obj["rank"] == rank, side
    rng = dict(obj["rng"])
    gens = rng.pop("generators", {})
    rng["numpy"] = _np_state_from_safe(rng["numpy"])
    py = rng["python"]
    rng["python"] = (py[0], tuple(py[1]), py[2])
    _set_rng_state(rng)
    for k, g in (generators or {}).items():
        if k in gens:
            g.set_state(gens[k])
    return True


def latest_resume(directory: str, name: str = "") -> Optional[str]:
    pats = glob.glob(os.path.join(directory, f"{name}*resume_*.pt"))
    best, best_step = None, -1
    for p in pats:
        m = re.search(r"resume_(\d+)\.pt$", p)
        if m and int(m.group(1)) > best_step:
            best, best_step = p, int(m.group(1))
    return best
