"""raft_stir_amd: MI355X-native RAFT optical-flow engine (PyTorch-ROCm + HIP/CDNA4 + RCCL).

Capabilities of athaddius/RAFT_STIR (RAFT / RAFT-small, all-pairs and
memory-efficient correlation, 4-stage training, Chairs/Sintel/KITTI
evaluation, STIR point-track TorchScript/ONNX export), re-designed for gfx950.
"""
__version__ = "0.1.0"

from .config import RAFTConfig, resolve_config, make_args  # noqa: F401


def __getattr__(name):
    if name == "RAFT":
        from .models.raft import RAFT
        return RAFT
    raise AttributeError(name)
