"""raft_stir_amd: MI355X-native RAFT optical-flow engine (PyTorch-ROCm + HIP/CDNA4 + RCCL).

Capabilities of athaddius/RAFT_STIR (RAFT / RAFT-small, all-pairs and
memory-efficient correlation, 4-stage training, Chairs/Sintel/KITTI
evaluation, STIR point-track TorchScript/ONNX export), re-designed for gfx950.
"""
__version__ = "0.1.0"

import os as _os

# MIOpen (the encoder convolutions) would otherwise run a ~20 s on-line
# solution search on the first call of every conv shape missing from its
# shipped find-db (measured: scripts/first_step_probe.py; the steady-state
# step time is the same or better in FAST mode).  Must be set before MIOpen
# initialises; a user setting wins.
_os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

from .config import RAFTConfig, resolve_config, make_args  # noqa: F401


def __getattr__(name):
    if name == "RAFT":
        from .models.raft import RAFT
        return RAFT
    raise AttributeError(name)
