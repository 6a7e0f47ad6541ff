import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_stir_amd.ops import _ext
    _ext.load(raise_on_error=True)  # a GPU test must never pass on a fallback
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def reference_raft():
    """The unmodified reference RAFT class (read-only import), or skip."""
    core = os.path.join(REFERENCE, "core")
    if not os.path.isdir(core):
        pytest.skip("reference not mounted")
    if core not in sys.path:
        sys.path.insert(0, core)
    import warnings
    warnings.filterwarnings("ignore")
    from raft import RAFT as RefRAFT  # noqa
    return RefRAFT


# ------------------------------------------------- fake dataset directory tree
import numpy as _np  # noqa: E402


def _write_img(path, h, w, seed):
    from PIL import Image
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(_np.random.RandomState(seed).randint(0, 255, (h, w, 3)).astype(_np.uint8)).save(path)


def _write_flo(path, h, w, seed):
    from raft_stir_amd.data import frame_utils as fu
    os.makedirs(os.path.dirname(path), exist_ok=True)
    fu.writeFlow(path, _np.random.RandomState(seed).randn(h, w, 2).astype(_np.float32))


@pytest.fixture(scope="session")
def fake_root(tmp_path_factory):
    """Tiny Chairs/Sintel/KITTI/HD1K/Things trees with the real layouts."""
    from PIL import Image
    from raft_stir_amd.data import frame_utils as fu
    np = _np
    root = tmp_path_factory.mktemp("datasets")
    H, W = 128, 160
    ch = root / "FlyingChairs_release" / "data"
    os.makedirs(ch)
    for i in range(3):
        Image.fromarray(np.random.RandomState(i).randint(0, 255, (H, W, 3)).astype(np.uint8)).save(ch / f"{i:05d}_img1.ppm")
        Image.fromarray(np.random.RandomState(10 + i).randint(0, 255, (H, W, 3)).astype(np.uint8)).save(ch / f"{i:05d}_img2.ppm")
        _write_flo(str(ch / f"{i:05d}_flow.flo"), H, W, i)
    np.savetxt(root / "FlyingChairs_release" / "chairs_split.txt", np.array([1, 2, 1]), fmt="%d")
    for split in ("training", "test"):
        for dst in ("clean", "final"):
            for s, scene in enumerate(("alley", "market")):
                for f in range(3):
                    _write_img(str(root / "Sintel" / split / dst / scene / f"frame_{f + 1:04d}.png"), H, W, s * 10 + f)
                    if split == "training" and f < 2 and dst == "clean":
                        _write_flo(str(root / "Sintel" / split / "flow" / scene / f"frame_{f + 1:04d}.flo"), H, W, f)
    for split in ("training", "testing"):
        for i in range(2):
            _write_img(str(root / "KITTI" / split / "image_2" / f"{i:06d}_10.png"), H, W, i)
            _write_img(str(root / "KITTI" / split / "image_2" / f"{i:06d}_11.png"), H, W, i + 5)
            if split == "training":
                os.makedirs(root / "KITTI" / split / "flow_occ", exist_ok=True)
                fl = np.random.RandomState(i).randn(H, W, 2) * 5
                fu.writeFlowKITTI(str(root / "KITTI" / split / "flow_occ" / f"{i:06d}_10.png"), fl)
    for f in range(3):
        _write_img(str(root / "HD1k" / "hd1k_input" / "image_2" / f"000000_{f:04d}.png"), H, W, f)
        os.makedirs(root / "HD1k" / "hd1k_flow_gt" / "flow_occ", exist_ok=True)
        fu.writeFlowKITTI(str(root / "HD1k" / "hd1k_flow_gt" / "flow_occ" / f"000000_{f:04d}.png"),
                          np.zeros((H, W, 2)))
    for dst in ("frames_cleanpass", "frames_finalpass"):
        for f in range(3):
            _write_img(str(root / "FlyingThings3D" / dst / "TRAIN" / "A" / "0000" / "left" / f"{f:04d}.png"), H, W, f)
    for d in ("into_future", "into_past"):
        for f in range(3):
            p = root / "FlyingThings3D" / "optical_flow" / "TRAIN" / "A" / "0000" / d / "left" / f"{f:04d}.pfm"
            os.makedirs(p.parent, exist_ok=True)
            fu.writePFM(str(p), np.random.RandomState(f).randn(H, W, 3).astype(np.float32))
    return root
