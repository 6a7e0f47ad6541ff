"""Data pipeline: file formats, native host ops, augmentors, datasets, loaders.

No datasets ship offline, so every dataset class is exercised on a tiny
synthetic directory tree laid out like the real one.  The native host ops
(_host.so: PNG codec, resize, jitter, sparse resize) are compared with the
pure-numpy fallbacks.  OpenCV/torchvision are not installed, so exact pixel
parity with cv2.resize / torchvision ColorJitter is "parity unpinned"; the
semantics (half-pixel-centre bilinear with edge clamp; PIL blend/HSV ops) are
pinned by the closed-form checks below.
"""
import os

import numpy as np
import pytest
import torch
from PIL import Image

from raft_stir_amd.data import augmentor as aug
from raft_stir_amd.data import datasets, frame_utils as fu


@pytest.fixture(scope="module", autouse=True)
def host_lib():
    from raft_stir_amd.build import build_host
    build_host()
    fu._HOST[0] = None
    assert fu._host_ops() is not None
    yield


def _no_host():
    class Ctx:
        def __enter__(self):
            self.prev = fu._HOST[0]
            fu._HOST[0] = False

        def __exit__(self, *a):
            fu._HOST[0] = self.prev
    return Ctx()


def test_flo_roundtrip(tmp_path):
    fl = np.random.RandomState(0).randn(13, 17, 2).astype(np.float32)
    p = str(tmp_path / "a.flo")
    fu.writeFlow(p, fl)
    assert np.array_equal(fu.readFlow(p), fl)
    fu.writeFlow(p, fl[..., 0], fl[..., 1])
    assert np.array_equal(fu.read_gen(p), fl)
    raw = open(p, "rb").read()
    assert np.frombuffer(raw[:4], "<f4")[0] == 202021.25
    assert tuple(np.frombuffer(raw[4:12], "<i4")) == (17, 13)


def test_flo_bad_magic(tmp_path):
    p = tmp_path / "bad.flo"
    p.write_bytes(b"\x00" * 32)
    assert fu.readFlow(str(p)) is None


def test_pfm_roundtrip_and_drop_third_channel(tmp_path):
    rs = np.random.RandomState(1)
    img3 = rs.randn(7, 9, 3).astype(np.float32)
    p = str(tmp_path / "a.pfm")
    fu.writePFM(p, img3)
    back = fu.readPFM(p)
    assert np.array_equal(back, img3)
    assert np.array_equal(fu.read_gen(p), img3[..., :2])
    gray = rs.randn(5, 4).astype(np.float32)
    fu.writePFM(p, gray)
    assert np.array_equal(fu.read_gen(p), gray)
    # big-endian variant (positive scale)
    with open(p, "wb") as f:
        f.write(b"Pf\n4 5\n1.0\n")
        f.write(np.flipud(gray).astype(">f4").tobytes())
    assert np.array_equal(fu.readPFM(p), gray)


@pytest.mark.parametrize("native", [True, False])
def test_kitti_png_roundtrip(tmp_path, native):
    rs = np.random.RandomState(2)
    fl = (rs.randn(11, 23, 2) * 20).astype(np.float32)
    p = str(tmp_path / "k.png")
    if native:
        fu.writeFlowKITTI(p, fl)
        flow, valid = fu.readFlowKITTI(p)
    else:
        with _no_host():
            fu.writeFlowKITTI(p, fl)
            flow, valid = fu.readFlowKITTI(p)
    assert np.abs(flow - fl).max() <= 1 / 64.0 + 1e-6
    assert (valid == 1).all()


def test_png_decoders_agree_with_pil(tmp_path):
    rs = np.random.RandomState(3)
    im8 = rs.randint(0, 255, (31, 45, 3)).astype(np.uint8)
    im8[:, :20] = 40  # make the encoder pick varied filters
    Image.fromarray(im8).save(tmp_path / "a.png", optimize=True)
    rgba = rs.randint(0, 255, (9, 10, 4)).astype(np.uint8)
    Image.fromarray(rgba, "RGBA").save(tmp_path / "b.png")
    g16 = rs.randint(0, 65535, (12, 14)).astype(np.uint16)
    Image.fromarray(g16).save(tmp_path / "c.png")
    for name, want in (("a.png", im8), ("b.png", rgba), ("c.png", g16[..., None])):
        data = open(tmp_path / name, "rb").read()
        nat = fu.png_read(str(tmp_path / name))
        pyd = fu._png_decode_numpy(data)
        assert np.array_equal(nat.astype(np.int64), want.astype(np.int64)), name
        assert np.array_equal(pyd.astype(np.int64), want.astype(np.int64)), name


def _png_bytes(tmp_path):
    rs = np.random.RandomState(5)
    im = rs.randint(0, 255, (17, 23, 3)).astype(np.uint8)
    Image.fromarray(im).save(tmp_path / "x.png")
    return open(tmp_path / "x.png", "rb").read()


def _chunk(typ, body):
    import struct
    import zlib
    return struct.pack(">I", len(body)) + typ + body + struct.pack(">I", zlib.crc32(typ + body) & 0xffffffff)


def test_png_corrupt_inputs_raise(tmp_path):
    """The native decoder parses untrusted files (reference: cv2.imread in
    core/utils/frame_utils.py:102-107): every malformed input must raise,
    never read out of bounds or allocate from a bogus header.  The same cases
    run under AddressSanitizer + UBSan in tests/test_sanitize_cpu.py."""
    import struct
    import zlib
    dec = fu._host_ops().png_decode

    def t(b):  # a fresh torch allocation of exactly len(b) bytes (ASan sees its bounds)
        return torch.tensor(np.frombuffer(bytes(b), np.uint8)) if len(b) else torch.empty(0, dtype=torch.uint8)
    good = _png_bytes(tmp_path)
    assert dec(t(good)).shape == (17, 23, 3)
    sig = good[:8]
    ihdr = lambda w, h, d=8, c=2: _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, d, c, 0, 0, 0))
    raw = zlib.compress(b"\x00" + b"\x01" * 9)
    cases = [good[:n] for n in (0, 5, 8, 12, 20, 33, 40, len(good) // 2, len(good) - 13)]
    cases += [
        sig + _chunk(b"IHDR", b"\x00\x00\x00\x03"),                          # short IHDR
        sig + ihdr(1 << 30, 1 << 30) + _chunk(b"IDAT", raw) + _chunk(b"IEND", b""),  # bogus huge size
        sig + ihdr(70000, 2) + _chunk(b"IDAT", raw) + _chunk(b"IEND", b""),
        sig + ihdr(3, 1) + _chunk(b"IDAT", b"not zlib at all") + _chunk(b"IEND", b""),
        sig + ihdr(3, 1) + _chunk(b"IDAT", zlib.compress(b"\x00\x01")) + _chunk(b"IEND", b""),  # short data
        sig + ihdr(3, 1) + _chunk(b"IDAT", zlib.compress(b"\x07" + b"\x01" * 9)) + _chunk(b"IEND", b""),  # filter 7
        sig + ihdr(3, 1, d=4) + _chunk(b"IDAT", raw) + _chunk(b"IEND", b""),  # bit depth 4
        sig + ihdr(3, 1, c=3) + _chunk(b"IDAT", raw) + _chunk(b"IEND", b""),  # palette
        sig + _chunk(b"IDAT", raw) + _chunk(b"IEND", b""),                      # no IHDR
        sig + struct.pack(">I", 0xFFFFFFF0) + b"IDAT",                         # chunk length past the end
    ]
    for i, c in enumerate(cases):
        with pytest.raises(RuntimeError):
            dec(t(c))
    # a valid file with one flipped byte either decodes or raises -- never crashes
    rs = np.random.RandomState(0)
    for _ in range(200):
        b = bytearray(good)
        b[rs.randint(8, len(b))] ^= 1 << rs.randint(8)
        try:
            dec(t(b))
        except RuntimeError:
            pass


def test_resize_semantics():
    # half-pixel centres + edge clamp: 2x upsampling of [0, 10] -> [0, 2.5, 7.5, 10]
    x = np.array([[0.0, 10.0]], np.float32)[..., None]
    up = aug._resize(x, 2.0, 1.0)[..., 0]
    assert np.allclose(up, [[0.0, 2.5, 7.5, 10.0]])
    rs = np.random.RandomState(4)
    for dt in (np.uint8, np.float32):
        img = (rs.rand(29, 37, 3) * 255).astype(dt)
        a = aug._resize(img, 1.31, 0.77)
        with _no_host():
            b = aug._resize(img, 1.31, 0.77)
        assert a.shape == b.shape == (int(round(29 * 0.77)), int(round(37 * 1.31)), 3)
        assert np.abs(a.astype(np.float64) - b.astype(np.float64)).max() <= (1 if dt == np.uint8 else 1e-4)


def test_jitter_native_matches_fallback_and_identity():
    rs = np.random.RandomState(5)
    img = rs.randint(0, 255, (20, 30, 3)).astype(np.uint8)
    assert np.array_equal(aug.apply_jitter(img, 1.0, 1.0, 1.0, 0.0, [0, 1, 2, 3]), img)
    for order in ([0, 1, 2, 3], [3, 1, 0, 2]):
        a = aug.apply_jitter(img, 1.3, 0.6, 1.4, -0.12, order)
        with _no_host():
            b = aug.apply_jitter(img, 1.3, 0.6, 1.4, -0.12, order)
        assert np.abs(a.astype(int) - b.astype(int)).max() <= 1
    # saturation 0 -> grey; brightness 0 -> black
    g = aug.apply_jitter(img, 1.0, 1.0, 0.0, 0.0, [2])
    assert (g[..., 0] == g[..., 1]).all() and (g[..., 1] == g[..., 2]).all()
    assert (aug.apply_jitter(img, 0.0, 1.0, 1.0, 0.0, [0]) == 0).all()


def test_sparse_resize_native_matches_fallback():
    rs = np.random.RandomState(6)
    flow = rs.randn(30, 40, 2).astype(np.float32)
    valid = (rs.rand(30, 40) > 0.7).astype(np.float32)
    a = aug.sparse_flow_resize(flow, valid, 1.3, 1.3)
    with _no_host():
        b = aug.sparse_flow_resize(flow, valid, 1.3, 1.3)
    assert np.allclose(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert a[1].sum() > 0 and np.allclose(a[0][a[1] == 0], 0)


def test_flow_augmentor_invariants():
    np.random.seed(0)
    torch.manual_seed(0)
    A = aug.FlowAugmentor(crop_size=[64, 96], min_scale=-0.2, max_scale=0.5)
    img1 = np.random.randint(0, 255, (120, 160, 3)).astype(np.uint8)
    img2 = np.random.randint(0, 255, (120, 160, 3)).astype(np.uint8)
    flow = np.ones((120, 160, 2), np.float32) * np.array([3.0, -2.0], np.float32)
    for _ in range(10):
        i1, i2, f = A(img1, img2, flow)
        assert i1.shape == i2.shape == (64, 96, 3) and f.shape == (64, 96, 2)
        assert i1.dtype == np.uint8 and f.dtype == np.float32
        # constant flow stays constant per component, scaled by |sx|,|sy| (signs flip with flips)
        assert np.allclose(f[..., 0], f[0, 0, 0], atol=1e-4)
        assert 3.0 * 0.5 < abs(f[0, 0, 0]) < 3.0 * 2.0


def test_sparse_augmentor_invariants():
    np.random.seed(1)
    torch.manual_seed(1)
    A = aug.SparseFlowAugmentor(crop_size=[48, 80], min_scale=-0.2, max_scale=0.4, do_flip=True)
    img = np.random.randint(0, 255, (90, 150, 3)).astype(np.uint8)
    flow = np.random.randn(90, 150, 2).astype(np.float32)
    valid = (np.random.rand(90, 150) > 0.5).astype(np.float32)
    flow[valid == 0] = 0  # KITTI convention: no flow where invalid
    for _ in range(10):
        i1, i2, f, v = A(img, img.copy(), flow, valid)
        assert i1.shape == (48, 80, 3) and f.shape == (48, 80, 2) and v.shape == (48, 80)
        assert np.allclose(f[v == 0], 0) and v.sum() > 0


def test_dataset_classes(fake_root):
    r = str(fake_root)
    chairs = datasets.FlyingChairs(split="training", root=f"{r}/FlyingChairs_release/data",
                                   split_file=f"{r}/FlyingChairs_release/chairs_split.txt")
    assert len(chairs) == 2
    assert len(datasets.FlyingChairs(split="train", root=f"{r}/FlyingChairs_release/data",
                                     split_file=f"{r}/FlyingChairs_release/chairs_split.txt")) == 2
    assert len(datasets.FlyingChairs(split="validation", root=f"{r}/FlyingChairs_release/data",
                                     split_file=f"{r}/FlyingChairs_release/chairs_split.txt")) == 1
    i1, i2, flow, valid = chairs[0]
    assert i1.shape == (3, 128, 160) and flow.shape == (2, 128, 160) and valid.shape == (128, 160)
    assert i1.dtype == torch.float32 and valid.max() == 1
    sintel = datasets.MpiSintel(split="training", root=f"{r}/Sintel", dstype="clean")
    assert len(sintel) == 4 and len(sintel.flow_list) == 4
    test = datasets.MpiSintel(split="test", root=f"{r}/Sintel", dstype="final")
    a, b, (scene, fid) = test[3]
    assert scene == "market" and fid == 1 and a.shape == (3, 128, 160)
    kitti = datasets.KITTI(split="training", root=f"{r}/KITTI")
    i1, i2, flow, valid = kitti[1]
    assert kitti.sparse and flow.shape == (2, 128, 160) and valid.sum() == 128 * 160
    things = datasets.FlyingThings3D(root=f"{r}/FlyingThings3D", dstype="frames_cleanpass")
    assert len(things) == 4
    i1, i2, flow, valid = things[0]
    assert flow.shape == (2, 128, 160)
    hd = datasets.HD1K(root=f"{r}/HD1k")
    assert len(hd) == 2
    rep = 3 * datasets.MpiSintel(split="training", root=f"{r}/Sintel", dstype="clean")
    assert len(rep) == 12


def test_fetch_dataloader_stages(fake_root):
    import argparse
    r = str(fake_root)
    for stage, size in (("chairs", [48, 64]), ("things", [48, 64]), ("sintel", [48, 64]),
                        ("kitti", [48, 64]), ("synthetic", [48, 64])):
        args = argparse.Namespace(stage=stage, image_size=size, batch_size=2, data_root=r,
                                  num_workers=0, chairs_split=f"{r}/FlyingChairs_release/chairs_split.txt",
                                  synthetic_length=8)
        loader = datasets.fetch_dataloader(args, rank=0, world_size=1, pin_memory=False)
        i1, i2, flow, valid = next(iter(loader))
        assert i1.shape == (2, 3, 48, 64) and flow.shape == (2, 2, 48, 64) and valid.shape == (2, 48, 64), stage


def test_worker_seeding_distinct(fake_root):
    import argparse
    args = argparse.Namespace(stage="synthetic", image_size=[32, 48], batch_size=2, num_workers=2,
                              synthetic_length=8)
    loader = datasets.fetch_dataloader(args, rank=0, world_size=1, pin_memory=False)
    batches = [b[0] for b in loader]
    assert len(batches) == 4


def test_flow_viz_wheel_and_image():
    from raft_stir_amd.utils import flow_viz
    wheel = flow_viz.make_colorwheel()
    assert wheel.shape == (55, 3)
    assert tuple(wheel[0]) == (255, 0, 0) and wheel.min() >= 0 and wheel.max() <= 255
    fl = np.zeros((4, 4, 2), np.float32)
    fl[0, 0] = [1, 0]
    img = flow_viz.flow_to_image(fl)
    assert img.shape == (4, 4, 3) and img.dtype == np.uint8
    assert tuple(img[1, 1]) == (255, 255, 255)  # zero flow -> white
    bgr = flow_viz.flow_to_image(fl, convert_to_bgr=True)
    assert np.array_equal(bgr[..., ::-1], img)


def test_packaged_chairs_split(tmp_path, monkeypatch):
    """Without a chairs_split.txt in the CWD or next to the data, FlyingChairs
    falls back to the packaged table: 22,872 pairs, 22,232 train / 640 val
    (SURVEY D3), identical to the reference file when it is present."""
    import os
    from raft_stir_amd.data.datasets import load_chairs_split
    monkeypatch.chdir(tmp_path)
    s = load_chairs_split("chairs_split.txt", str(tmp_path / "nodata"))
    assert s.shape == (22872,) and (s == 1).sum() == 22232 and (s == 2).sum() == 640
    ref = "/root/reference/chairs_split.txt"
    if os.path.exists(ref):
        assert np.array_equal(s, np.loadtxt(ref, dtype=np.int32))


def test_packaged_chairs_split_rejects_other_release(fake_root, tmp_path, monkeypatch):
    """A Chairs copy whose pair count differs from the packaged table's 22,872
    fails loudly instead of mislabelling train / validation pairs."""
    monkeypatch.chdir(tmp_path)
    with pytest.raises(ValueError, match="has 22872 entries but .* holds 3 flow files"):
        datasets.FlyingChairs(split="training", root=f"{fake_root}/FlyingChairs_release/data",
                              split_file="no_such_split.txt")


def test_fused_resize_crop_matches_resize_then_crop(monkeypatch):
    """FlowAugmentor.spatial_transform's native crop-window resize
    (csrc_host resize_crop) is bitwise the full resize + flips + crop."""
    from raft_stir_amd.data import frame_utils
    rs = np.random.RandomState(7)
    img1 = rs.randint(0, 255, (96, 128, 3)).astype(np.uint8)
    img2 = rs.randint(0, 255, (96, 128, 3)).astype(np.uint8)
    flow = rs.randn(96, 128, 2).astype(np.float32) * 5
    a = aug.FlowAugmentor((64, 80), min_scale=-0.2, max_scale=0.8, do_flip=True)
    a.h_flip_prob = a.v_flip_prob = 0.5
    ops = frame_utils._host_ops()
    if ops is None or not hasattr(ops, "resize_crop"):
        pytest.skip("native host ops not built")

    class NoFused:  # the host ops minus resize_crop
        def __getattr__(self, k):
            if k == "resize_crop":
                raise AttributeError(k)
            return getattr(ops, k)
    for seed in range(12):
        np.random.seed(seed)
        got = a.spatial_transform(img1, img2, flow)
        monkeypatch.setattr(aug, "_host_ops", lambda: NoFused())
        np.random.seed(seed)
        want = a.spatial_transform(img1, img2, flow)
        monkeypatch.undo()
        for g, w in zip(got, want):
            assert g.shape == w.shape and np.array_equal(np.ascontiguousarray(g), np.ascontiguousarray(w)), seed


def test_auto_workers_share_the_cpus(monkeypatch):
    """DataLoader workers per rank: up to FEED_WORKERS, within this process's
    CPU share (affinity / local ranks, one CPU kept for the trainer)."""
    from raft_stir_amd.data import datasets as D
    monkeypatch.setattr(D.os, "sched_getaffinity", lambda pid: set(range(64)))
    assert D.auto_workers(1) == D.FEED_WORKERS
    assert D.auto_workers(8) == 7
    monkeypatch.setattr(D.os, "sched_getaffinity", lambda pid: {0})
    assert D.auto_workers(1) == 0
