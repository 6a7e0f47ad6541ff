"""Flow / image file I/O (reference core/utils/frame_utils.py, same API).

* ``readFlow`` / ``writeFlow``: Middlebury ``.flo`` -- float32 magic 202021.25,
  int32 width, int32 height, then interleaved float32 (u, v) rows
  (reference frame_utils.py:12-31, 70-99).  Explicit little-endian dtypes, so
  it is also correct on big-endian hosts (the reference's warning at :17).
* ``readPFM``: ``PF``/``Pf`` header, endianness from the sign of the scale,
  rows stored bottom-up (reference :33-68).
* ``readFlowKITTI`` / ``writeFlowKITTI`` / ``readDispKITTI``: 16-bit PNGs,
  flow = (v - 2^15) / 64, valid in the third channel (reference :102-120).
  OpenCV is not available on this platform; the 16-bit PNG codec is the
  engine's own native one (csrc_host/dataops.cpp, zlib), with a pure-numpy
  decoder as the fallback when ``_host.so`` is not built.
* ``read_gen``: dispatch on the file extension (reference :123-137).
"""
from __future__ import annotations

import os
import re
import struct
import zlib
from os.path import splitext

import numpy as np
from PIL import Image

TAG_FLOAT = 202021.25
TAG_CHAR = np.array([TAG_FLOAT], np.float32)

_HOST = [None]


def _host_ops():
    """torch.ops.raft_stir_host if _host.so is built, else None."""
    if _HOST[0] is None:
        try:
            import torch
            path = os.environ.get("RAFT_STIR_HOST_LIB") or os.path.join(
                os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_host.so")
            if os.path.exists(path) and os.environ.get("RAFT_STIR_NO_HOST") != "1":
                torch.ops.load_library(path)
                _HOST[0] = torch.ops.raft_stir_host
            else:
                _HOST[0] = False
        except Exception:
            _HOST[0] = False
    return _HOST[0] or None


# ------------------------------------------------------------------ .flo
def readFlow(fn):
    """Read a Middlebury .flo file -> (H, W, 2) float32, or None on a bad magic."""
    with open(fn, "rb") as f:
        magic = np.fromfile(f, "<f4", count=1)
        if magic.size != 1 or magic[0] != TAG_FLOAT:
            print("Magic number incorrect. Invalid .flo file")
            return None
        w = int(np.fromfile(f, "<i4", count=1)[0])
        h = int(np.fromfile(f, "<i4", count=1)[0])
        data = np.fromfile(f, "<f4", count=2 * w * h)
    return np.resize(data, (h, w, 2)).astype(np.float32)


def writeFlow(filename, uv, v=None):
    """Write a .flo file from (H, W, 2) ``uv`` or separate ``uv`` (=u), ``v``."""
    if v is None:
        assert uv.ndim == 3 and uv.shape[2] == 2
        u, v = uv[:, :, 0], uv[:, :, 1]
    else:
        u = uv
    assert u.shape == v.shape
    h, w = u.shape
    inter = np.empty((h, w, 2), "<f4")
    inter[..., 0] = u
    inter[..., 1] = v
    with open(filename, "wb") as f:
        f.write(TAG_CHAR.astype("<f4").tobytes())
        f.write(np.array([w, h], "<i4").tobytes())
        f.write(inter.tobytes())


# ------------------------------------------------------------------ PFM
def readPFM(file):
    with open(file, "rb") as f:
        header = f.readline().rstrip()
        if header == b"PF":
            color = True
        elif header == b"Pf":
            color = False
        else:
            raise Exception("Not a PFM file.")
        m = re.match(rb"^(\d+)\s(\d+)\s$", f.readline())
        if not m:
            raise Exception("Malformed PFM header.")
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.fromfile(f, endian + "f")
    shape = (height, width, 3) if color else (height, width)
    return np.flipud(np.reshape(data, shape))


def writePFM(file, image, scale=1.0):
    """Little-endian PFM writer (for tests and tooling)."""
    image = np.asarray(image, dtype=np.float32)
    color = image.ndim == 3 and image.shape[2] == 3
    with open(file, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(b"%d %d\n" % (image.shape[1], image.shape[0]))
        f.write(b"%f\n" % (-abs(scale)))
        f.write(np.flipud(image).astype("<f4").tobytes())


# ------------------------------------------------------------ PNG (16-bit)
def _paeth_row(raw, prev, bpp):
    out = np.empty_like(raw)
    n = raw.shape[0]
    for i in range(n):
        a = int(out[i - bpp]) if i >= bpp else 0
        b = int(prev[i])
        c = int(prev[i - bpp]) if i >= bpp else 0
        p = a + b - c
        pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
        pred = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
        out[i] = (int(raw[i]) + pred) & 255
    return out


def _png_decode_numpy(data: bytes) -> np.ndarray:
    """Pure-numpy PNG decoder (8/16-bit, non-interlaced, non-palette). Slow
    for Paeth rows; used only when the native codec is not built."""
    assert data[:8] == b"\x89PNG\r\n\x1a\n", "not a PNG"
    off, idat = 8, []
    w = h = depth = ctype = None
    while off < len(data):
        (ln,) = struct.unpack(">I", data[off:off + 4])
        typ = data[off + 4:off + 8]
        body = data[off + 8:off + 8 + ln]
        if typ == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            assert body[12] == 0, "interlaced PNG unsupported"
        elif typ == b"IDAT":
            idat.append(body)
        elif typ == b"IEND":
            break
        off += 12 + ln
    C = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    bps = depth // 8
    bpp = C * bps
    stride = w * bpp
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8).reshape(h, stride + 1)
    img = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.uint8)
    for y in range(h):
        f, row = raw[y, 0], raw[y, 1:]
        if f == 0:
            cur = row.copy()
        elif f == 1:
            cur = row.astype(np.int64).reshape(-1, bpp).cumsum(0).reshape(-1).astype(np.uint8)
        elif f == 2:
            cur = (row.astype(np.int64) + prev).astype(np.uint8)
        elif f == 3:
            cur = np.empty(stride, np.uint8)
            for i in range(stride):
                a = int(cur[i - bpp]) if i >= bpp else 0
                cur[i] = (int(row[i]) + ((a + int(prev[i])) >> 1)) & 255
        else:
            cur = _paeth_row(row, prev, bpp)
        img[y] = cur
        prev = cur
    if depth == 16:
        return img.reshape(h, w * C, 2).astype(np.uint16).dot(np.array([256, 1], np.uint16)) \
            .reshape(h, w, C).astype(np.int32)
    return img.reshape(h, w, C)


def png_read(filename) -> np.ndarray:
    """Decode a PNG -> (H, W, C); 16-bit images as int32 (values 0..65535)."""
    with open(filename, "rb") as f:
        data = f.read()
    ops = _host_ops()
    if ops is not None:
        import torch
        return ops.png_decode(torch.frombuffer(bytearray(data), dtype=torch.uint8)).numpy()
    return _png_decode_numpy(data)


def png_write16(filename, img) -> None:
    """Encode (H, W, C) values 0..65535 as a 16-bit PNG."""
    img = np.ascontiguousarray(np.asarray(img).astype(np.int32))
    ops = _host_ops()
    if ops is not None:
        import torch
        data = ops.png_encode16(torch.from_numpy(img)).numpy().tobytes()
    else:
        h, w, c = img.shape
        be = np.clip(img, 0, 65535).astype(">u2").reshape(h, w * c)
        raw = b"".join(b"\x00" + be[y].tobytes() for y in range(h))
        ctype = {1: 0, 2: 4, 3: 2, 4: 6}[c]

        def chunk(t, b):
            return struct.pack(">I", len(b)) + t + b + struct.pack(">I", zlib.crc32(t + b))
        data = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 16, ctype, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))
    with open(filename, "wb") as f:
        f.write(data)


# ------------------------------------------------------------------ KITTI
def readFlowKITTI(filename):
    """KITTI flow PNG -> (flow (H,W,2) float32, valid (H,W) float32).

    The file stores (u, v, valid) in its R, G, B channels (OpenCV's BGR read
    followed by ``[..., ::-1]`` in the reference yields the same order)."""
    img = png_read(filename).astype(np.float32)
    flow, valid = img[:, :, :2], img[:, :, 2]
    flow = (flow - 2 ** 15) / 64.0
    return flow, valid


def readDispKITTI(filename):
    disp = png_read(filename)[..., 0].astype(np.float32) / 256.0
    valid = disp > 0.0
    flow = np.stack([-disp, np.zeros_like(disp)], -1)
    return flow, valid


def writeFlowKITTI(filename, uv):
    uv = 64.0 * np.asarray(uv, np.float64) + 2 ** 15
    valid = np.ones([uv.shape[0], uv.shape[1], 1])
    png_write16(filename, np.concatenate([uv, valid], axis=-1).astype(np.uint16))


# ------------------------------------------------------------------ generic
def read_gen(file_name, pil=False):
    ext = splitext(file_name)[-1].lower()
    if ext in (".png", ".jpeg", ".ppm", ".jpg"):
        return Image.open(file_name)
    if ext in (".bin", ".raw"):
        return np.load(file_name)  # allow_pickle=False (numpy default)
    if ext == ".flo":
        return readFlow(file_name).astype(np.float32)
    if ext == ".pfm":
        flow = readPFM(file_name).astype(np.float32)
        return flow if flow.ndim == 2 else flow[:, :, :-1]
    return []
