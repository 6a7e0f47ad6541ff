"""Evaluation, submissions, STIR export and the root CLI scripts, on CPU with
tiny fake datasets (no dataset or checkpoint ships offline)."""
import argparse
import glob
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from raft_stir_amd.config import make_args
from raft_stir_amd.eval import evaluate as ev
from raft_stir_amd.models import RAFT

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def small_model():
    torch.manual_seed(0)
    return RAFT(make_args(small=True)).eval()


def test_validate_all(fake_root, small_model):
    r = str(fake_root)
    res = ev.validate_chairs(small_model, iters=2, root=f"{r}/FlyingChairs_release/data",
                             split_file=f"{r}/FlyingChairs_release/chairs_split.txt")
    assert set(res) == {"chairs"} and np.isfinite(res["chairs"])
    res = ev.validate_sintel(small_model, iters=2, root=f"{r}/Sintel")
    assert set(res) == {"clean", "final"}  # both passes share training/flow
    res = ev.validate_kitti(small_model, iters=2, root=f"{r}/KITTI")
    assert set(res) == {"kitti-epe", "kitti-f1"} and 0 <= res["kitti-f1"] <= 100


def test_chairs_empty_root_raises(tmp_path, small_model):
    (tmp_path / "split.txt").write_text("")
    with pytest.raises(FileNotFoundError):
        ev.validate_chairs(small_model, iters=2, root=str(tmp_path / "none"), split_file=str(tmp_path / "split.txt"))


def test_chairs_epe_matches_manual(fake_root, small_model):
    from raft_stir_amd.data import datasets
    r = str(fake_root)
    kw = dict(root=f"{r}/FlyingChairs_release/data", split_file=f"{r}/FlyingChairs_release/chairs_split.txt")
    ds = datasets.FlyingChairs(split="validation", **kw)
    i1, i2, gt, _ = ds[0]
    with torch.no_grad():
        _, up = small_model(i1[None], i2[None], iters=2, test_mode=True)
    want = torch.sum((up[0] - gt) ** 2, dim=0).sqrt().mean().item()
    got = ev.validate_chairs(small_model, iters=2, **kw)["chairs"]
    assert abs(got - want) < 1e-4


def test_submissions(fake_root, small_model, tmp_path):
    from raft_stir_amd.data import frame_utils as fu
    r = str(fake_root)
    ev.create_sintel_submission(small_model, iters=2, warm_start=True, root=f"{r}/Sintel",
                                output_path=str(tmp_path / "sintel"))
    flos = sorted(glob.glob(str(tmp_path / "sintel" / "*" / "*" / "*.flo")))
    assert len(flos) == 8  # 2 passes x 2 scenes x 2 pairs
    assert fu.readFlow(flos[0]).shape == (128, 160, 2)
    ev.create_kitti_submission(small_model, iters=2, root=f"{r}/KITTI", output_path=str(tmp_path / "kitti"))
    pngs = sorted(glob.glob(str(tmp_path / "kitti" / "*.png")))
    assert len(pngs) == 2
    flow, valid = fu.readFlowKITTI(pngs[0])
    assert flow.shape == (128, 160, 2) and (valid == 1).all()


def test_pointtrack_semantics_and_torchscript(small_model, tmp_path):
    from raft_stir_amd.export.pointtrack import RaftPointTrack, export_pointtrack
    tracker = RaftPointTrack(small_model, iters=3)
    g = torch.Generator().manual_seed(0)
    i1, i2 = torch.rand(1, 3, 128, 160, generator=g) * 255, torch.rand(1, 3, 128, 160, generator=g) * 255
    pts = torch.tensor([[[0.0, 0.0], [159.0, 127.0], [10.0, 20.0]]])
    with torch.no_grad():
        end = tracker(pts, i1, i2)
        _, up = small_model(i1, i2, iters=3, test_mode=True)
    assert end.shape == (1, 3, 2)
    # integer points sample the flow exactly (align_corners=True)
    torch.testing.assert_close(end[0, 0], pts[0, 0] + up[0, :, 0, 0])
    torch.testing.assert_close(end[0, 1], pts[0, 1] + up[0, :, 127, 159])
    torch.testing.assert_close(end[0, 2], pts[0, 2] + up[0, :, 20, 10])
    out = export_pointtrack(small_model, str(tmp_path / "pt"), size=(128, 160), npoints=32, iters=3)
    loaded = torch.jit.load(out["torchscript"])
    pts = torch.rand(1, 32, 2, generator=g) * 120
    with torch.no_grad():
        torch.testing.assert_close(loaded(pts, i1, i2), tracker(pts, i1, i2), atol=1e-3, rtol=1e-3)
    graph = str(loaded.inlined_graph)
    assert "raft_stir::" not in graph and "grid_sampler" in graph  # standard ops only


def test_cli_scripts(fake_root, tmp_path):
    r = str(fake_root)
    env = dict(os.environ, PYTHONPATH=ROOT)
    frames = sorted(glob.glob(f"{r}/Sintel/training/clean/alley/*.png"))
    res = subprocess.run([sys.executable, os.path.join(ROOT, "demo.py"), "--small", "--path",
                          os.path.dirname(frames[0]), "--iters", "2", "--out", str(tmp_path / "demo"),
                          "--model", str(tmp_path / "missing.pth"), "--random_init"],
                         env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0, res.stderr[-2000:]
    assert len(glob.glob(str(tmp_path / "demo" / "*_flow.png"))) == 2
    res = subprocess.run([sys.executable, os.path.join(ROOT, "evaluate.py"), "--small", "--dataset", "kitti",
                          "--data_root", r, "--iters", "2", "--random_init"], env=env, capture_output=True, text=True, timeout=600)
    assert res.returncode == 0 and "Validation KITTI" in res.stdout, res.stderr[-2000:]
    res = subprocess.run([sys.executable, os.path.join(ROOT, "rafttoonnx.py"), "--path", os.path.dirname(frames[0]),
                          "--model", str(tmp_path / "missing.pth"), "--random_init", "--out", str(tmp_path / "exp")],
                         env=env, capture_output=True, text=True, timeout=900)
    assert res.returncode == 0, res.stderr[-2000:]
    assert os.path.exists(tmp_path / "exp" / "raft_pointtrackSTIR.pt")
    # the demo-shape export of the bare model (ONNX, or TorchScript without onnx)
    assert os.path.exists(tmp_path / "exp" / "raftsmall.pt") or os.path.exists(tmp_path / "exp" / "raftsmall.onnx")
    # ... and the STIR-shape (1x3x512x640) bare-model export, reference rafttoonnx.py:94-118
    assert (os.path.exists(tmp_path / "exp" / "raftsmall_STIR.pt")
            or os.path.exists(tmp_path / "exp" / "raftsmall_STIR.onnx"))
    if not os.path.exists(tmp_path / "exp" / "raftsmall_STIR.onnx"):
        assert "raftsmall_STIR.pt (TorchScript, max|diff| vs eager" in res.stdout
    # without --random_init a missing checkpoint is an error (reference CLIs load strictly)
    res = subprocess.run([sys.executable, os.path.join(ROOT, "evaluate.py"), "--small", "--dataset", "kitti",
                          "--data_root", r, "--model", str(tmp_path / "typo.pth")], env=env,
                         capture_output=True, text=True, timeout=600)
    assert res.returncode != 0 and "typo.pth" in res.stderr


def test_core_shim_imports():
    # another test may have imported the reference's own core/raft.py as 'raft'
    saved = {k: sys.modules.pop(k) for k in ("raft", "utils.utils", "utils") if k in sys.modules}
    sys.path.insert(0, os.path.join(ROOT, "core"))
    try:
        import importlib
        raft = importlib.import_module("raft")
        utils_utils = importlib.import_module("utils.utils")
        assert raft.RAFT is RAFT
        assert hasattr(utils_utils, "InputPadder") and hasattr(utils_utils, "forward_interpolate")
    finally:
        sys.path.remove(os.path.join(ROOT, "core"))
        for k in ("raft", "utils.utils", "utils"):
            sys.modules.pop(k, None)
        sys.modules.update(saved)


def test_shipped_demo_frames():
    """demo-frames/ (scripts/make_demo_frames.py) is the default --path of
    demo.py / rafttoonnx.py: procedural frames with a known motion."""
    import importlib.util
    import numpy as np
    from raft_stir_amd.data import frame_utils
    frames = sorted(glob.glob(os.path.join(ROOT, "demo-frames", "*.png")))
    assert len(frames) >= 2
    img = np.asarray(frame_utils.read_gen(frames[0]))
    assert img.shape == (436, 1024, 3) and img.dtype == np.uint8
    spec = importlib.util.spec_from_file_location("mdf", os.path.join(ROOT, "scripts", "make_demo_frames.py"))
    mdf = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mdf)
    assert np.array_equal(mdf.frame(0), img)  # regenerates bit-identically
    # the background moves by (3, 1) px: frame 1 == frame 0 shifted, away from the disk
    f0, f1 = mdf.frame(0).astype(int), mdf.frame(1).astype(int)
    assert np.abs(f1[11:100, 13:300] - f0[10:99, 10:297]).max() <= 1
