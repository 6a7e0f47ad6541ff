"""raft_stir_amd: MI355X-native RAFT optical-flow engine (PyTorch-ROCm + HIP/CDNA4 + RCCL).

Capabilities of athaddius/RAFT_STIR (RAFT / RAFT-small, all-pairs and
memory-efficient correlation, 4-stage training, Chairs/Sintel/KITTI
evaluation, STIR point-track TorchScript/ONNX export), re-designed for gfx950.
"""
__version__ = "0.1.0"

import os as _os

# MIOpen (the encoder convolutions) runs an on-line solution search (~20 s)
# on the first call of every conv shape missing from its shipped find-db.
# The results of that search on MI355X for this model's shapes are kept in
# the package (miopen_db/, a text find-db written by MIOpen itself), so a
# fresh process starts with them.  MIOPEN_FIND_MODE=FAST is NOT an option:
# its fallback picks CK weight-gradient kernels ~50x slower (535 ms/step vs
# 39 ms measured).  A user setting wins; must be set before MIOpen starts.
_os.environ.setdefault("MIOPEN_USER_DB_PATH",
                       _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "miopen_db"))
# kernel arguments in device memory: this step issues ~700 launches; with
# HIP_FORCE_DEV_KERNARG=0 the headline step measured 19.2 vs 18.3 ms and the
# graphed inference 3.31 vs 2.98 ms (profiles/r6/ab_dev_kernarg_s40.txt).
# Pinned here in case an environment turns it off; read at HIP start-up.
_os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")

from .config import RAFTConfig, resolve_config, make_args  # noqa: F401


def __getattr__(name):
    if name == "RAFT":
        from .models.raft import RAFT
        return RAFT
    raise AttributeError(name)
