"""Training-time augmentation (reference core/utils/augmentor.py, same API and
parameters).

``FlowAugmentor(crop_size, min_scale=-0.2, max_scale=0.5, do_flip=True)``
    colour jitter (brightness/contrast/saturation 0.4, hue 0.5/pi; asymmetric
    with p=0.2, otherwise the pair is jittered as one stacked image), eraser
    (p=0.5, 1-2 boxes of 50-100 px filled with img2's mean colour), random
    scale 2^U(min,max) with stretch (p=0.8, +-0.2 octave) applied with
    p=0.8 (bilinear; flow multiplied by the scale), h-flip 0.5 / v-flip 0.1,
    random crop (reference augmentor.py:15-120).
``SparseFlowAugmentor(crop_size, min_scale=-0.2, max_scale=0.5, do_flip=False)``
    symmetric jitter 0.3 / hue 0.3/pi, eraser, scale with sparse scatter
    resize of flow+valid, h-flip only, crop with y/x margins 20/50
    (reference augmentor.py:122-246).

Random draws use numpy's global RNG for geometry and torch's RNG for the
jitter factors (as torchvision does), so per-worker seeding
(datasets.FlowDataset) reproduces streams.  The pixel kernels (bilinear
resize with OpenCV INTER_LINEAR semantics, PIL-semantics colour jitter, sparse
flow scatter) are the engine's native host ops (csrc_host/dataops.cpp); numpy
fallbacks keep the module importable without ``_host.so``.
"""
from __future__ import annotations

import numpy as np
import torch

from .frame_utils import _host_ops


# ------------------------------------------------------------- primitives
def _resize(img: np.ndarray, fx: float, fy: float) -> np.ndarray:
    h, w = img.shape[:2]
    oh, ow = int(round(h * fy)), int(round(w * fx))
    ops = _host_ops()
    if ops is not None:
        t = torch.from_numpy(np.ascontiguousarray(img))
        if t.dtype not in (torch.uint8, torch.float32):
            t = t.float()
        return ops.resize_bilinear(t, oh, ow, fy, fx).numpy()
    return _resize_numpy(img, oh, ow, fy, fx)


def _resize_numpy(img, oh, ow, fy, fx):
    h, w = img.shape[:2]

    def taps(n_in, n_out, s):
        d = (np.arange(n_out) + 0.5) / s - 0.5
        i0 = np.floor(d).astype(np.int64)
        w1 = (d - i0).astype(np.float32)
        w1[i0 < 0] = 0
        i0 = np.clip(i0, 0, n_in - 1)
        w1[i0 >= n_in - 1] = 0
        i1 = np.minimum(i0 + 1, n_in - 1)
        return i0, i1, w1

    y0, y1, wy = taps(h, oh, fy)
    x0, x1, wx = taps(w, ow, fx)
    f = img.astype(np.float32)
    if f.ndim == 2:
        f = f[..., None]
    r0 = f[y0][:, x0] + wx[None, :, None] * (f[y0][:, x1] - f[y0][:, x0])
    r1 = f[y1][:, x0] + wx[None, :, None] * (f[y1][:, x1] - f[y1][:, x0])
    out = r0 + wy[:, None, None] * (r1 - r0)
    if img.ndim == 2:
        out = out[..., 0]
    if img.dtype == np.uint8:
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    return out


class ColorJitter:
    """torchvision.transforms.ColorJitter(brightness, contrast, saturation, hue)
    semantics on uint8 HxWx3 arrays: factors uniform in [max(0,1-x), 1+x],
    hue in [-h, h], the four operations in a random order."""

    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.0):
        self.b = (max(0.0, 1 - brightness), 1 + brightness)
        self.c = (max(0.0, 1 - contrast), 1 + contrast)
        self.s = (max(0.0, 1 - saturation), 1 + saturation)
        self.h = (-hue, hue)

    def sample(self):
        order = torch.randperm(4).tolist()
        u = lambda lo_hi: float(torch.empty(1).uniform_(lo_hi[0], lo_hi[1]))
        return order, u(self.b), u(self.c), u(self.s), u(self.h)

    def __call__(self, img: np.ndarray) -> np.ndarray:
        order, b, c, s, h = self.sample()
        return apply_jitter(img, b, c, s, h, order)


def apply_jitter(img, b, c, s, h, order):
    ops = _host_ops()
    if ops is not None:
        return ops.color_jitter(torch.from_numpy(np.ascontiguousarray(img)), b, c, s, h,
                                order).numpy()
    x = img.astype(np.float32)
    luma = lambda a: np.floor((a[..., 0] * 19595 + a[..., 1] * 38470 + a[..., 2] * 7471 + 0x8000)
                              / 65536.0)
    for op in order:
        if op == 0:
            x = np.clip(x * b, 0, 255).astype(np.uint8).astype(np.float32)
        elif op == 1:
            m = float(int(luma(x).mean() + 0.5))
            x = np.clip(m + c * (x - m), 0, 255).astype(np.uint8).astype(np.float32)
        elif op == 2:
            g = luma(x)[..., None]
            x = np.clip(g + s * (x - g), 0, 255).astype(np.uint8).astype(np.float32)
        elif op == 3 and h != 0.0:
            x = _hue_shift(x, h)
    return x.astype(np.uint8)


def _hue_shift(x, hue):
    r, g, b = x[..., 0], x[..., 1], x[..., 2]
    mx, mn = x.max(-1), x.min(-1)
    d = np.where(mx > mn, mx - mn, 1.0)
    rc, gc, bc = (mx - r) / d, (mx - g) / d, (mx - b) / d
    hh = np.where(r == mx, bc - gc, np.where(g == mx, 2 + rc - bc, 4 + gc - rc)) / 6.0
    hh = hh - np.floor(hh)
    hq = np.where(mx > mn, np.floor(hh * 255), 0).astype(np.int64)
    sq = np.where(mx > mn, np.floor((mx - mn) / np.maximum(mx, 1) * 255), 0)
    hq = (hq + int(hue * 255)) & 255
    hf, sf, v = hq / 255.0, sq / 255.0, mx
    i = np.floor(hf * 6)
    f = hf * 6 - i
    p, q, t = np.rint(v * (1 - sf)), np.rint(v * (1 - sf * f)), np.rint(v * (1 - sf * (1 - f)))
    i = i.astype(np.int64) % 6
    sel = [np.stack(c, -1) for c in ((v, t, p), (q, v, p), (p, v, t), (p, q, v), (t, p, v), (v, p, q))]
    out = np.zeros_like(x)
    for k in range(6):
        out = np.where((i == k)[..., None], sel[k], out)
    out = np.where((sf == 0)[..., None], np.stack([v, v, v], -1), out)
    return out


def sparse_flow_resize(flow, valid, fx=1.0, fy=1.0):
    ops = _host_ops()
    if ops is not None:
        f, v = ops.sparse_flow_resize(torch.from_numpy(np.ascontiguousarray(flow, np.float32)),
                                      torch.from_numpy(np.ascontiguousarray(valid, np.float32)),
                                      fx, fy)
        return f.numpy(), v.numpy()
    ht, wd = flow.shape[:2]
    xs, ys = np.meshgrid(np.arange(wd), np.arange(ht))
    coords = np.stack([xs, ys], -1).reshape(-1, 2).astype(np.float32)
    fl = flow.reshape(-1, 2).astype(np.float32)
    vv = valid.reshape(-1).astype(np.float32)
    c0, f0 = coords[vv >= 1], fl[vv >= 1]
    ht1, wd1 = int(round(ht * fy)), int(round(wd * fx))
    c1 = c0 * np.array([fx, fy], np.float32)
    f1 = f0 * np.array([fx, fy], np.float32)
    xx = np.round(c1[:, 0]).astype(np.int32)
    yy = np.round(c1[:, 1]).astype(np.int32)
    ok = (xx > 0) & (xx < wd1) & (yy > 0) & (yy < ht1)
    flow_img = np.zeros([ht1, wd1, 2], np.float32)
    valid_img = np.zeros([ht1, wd1], np.int32)
    flow_img[yy[ok], xx[ok]] = f1[ok]
    valid_img[yy[ok], xx[ok]] = 1
    return flow_img, valid_img


def _erase(img1, img2, prob, bounds=(50, 100)):
    ht, wd = img1.shape[:2]
    if np.random.rand() < prob:
        img2 = img2.copy()
        mean_color = img2.reshape(-1, 3).sum(0, dtype=np.int64) / (img2.size // 3)
        for _ in range(np.random.randint(1, 3)):
            x0 = np.random.randint(0, wd)
            y0 = np.random.randint(0, ht)
            dx = np.random.randint(bounds[0], bounds[1])
            dy = np.random.randint(bounds[0], bounds[1])
            img2[y0:y0 + dy, x0:x0 + dx, :] = mean_color
    return img1, img2


# ------------------------------------------------------------ augmentors
class FlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=True):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.4, contrast=0.4, saturation=0.4, hue=0.5 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        if np.random.rand() < self.asymmetric_color_aug_prob:
            return self.photo_aug(img1), self.photo_aug(img2)
        stack = self.photo_aug(np.concatenate([img1, img2], axis=0))
        return tuple(np.split(stack, 2, axis=0))

    def eraser_transform(self, img1, img2, bounds=(50, 100)):
        return _erase(img1, img2, self.eraser_aug_prob, bounds)

    def spatial_transform(self, img1, img2, flow):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 8) / float(ht),
                               (self.crop_size[1] + 8) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = scale_y = scale
        if np.random.rand() < self.stretch_prob:
            scale_x *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
            scale_y *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
        scale_x = float(np.clip(scale_x, min_scale, None))
        scale_y = float(np.clip(scale_y, min_scale, None))
        # the draws in the reference's order (scale, stretch, resize?, flips,
        # crop); the crop offsets depend only on the resized SIZE, so the
        # native path resizes just the crop window (csrc_host resize_crop)
        resize = np.random.rand() < self.spatial_aug_prob
        hflip = vflip = False
        if self.do_flip:
            hflip = np.random.rand() < self.h_flip_prob
            vflip = np.random.rand() < self.v_flip_prob
        oh, ow = (int(round(ht * scale_y)), int(round(wd * scale_x))) if resize else (ht, wd)
        y0 = np.random.randint(0, oh - self.crop_size[0])
        x0 = np.random.randint(0, ow - self.crop_size[1])
        ch, cw = self.crop_size
        ops = _host_ops()
        if resize and ops is not None and hasattr(ops, "resize_crop"):
            sgn = (-1.0 if hflip else 1.0, -1.0 if vflip else 1.0)
            rc = lambda a, mul: ops.resize_crop(torch.from_numpy(np.ascontiguousarray(a)), oh, ow, scale_y, scale_x,
                                                int(y0), int(x0), ch, cw, hflip, vflip, mul).numpy()
            return (rc(img1, []), rc(img2, []),
                    rc(flow.astype(np.float32), [scale_x * sgn[0], scale_y * sgn[1]]))
        if resize:
            img1 = _resize(img1, scale_x, scale_y)
            img2 = _resize(img2, scale_x, scale_y)
            flow = _resize(flow.astype(np.float32), scale_x, scale_y)
            flow = flow * np.array([scale_x, scale_y], np.float32)
        if hflip:
            img1, img2 = img1[:, ::-1], img2[:, ::-1]
            flow = flow[:, ::-1] * np.array([-1.0, 1.0], np.float32)
        if vflip:
            img1, img2 = img1[::-1, :], img2[::-1, :]
            flow = flow[::-1, :] * np.array([1.0, -1.0], np.float32)
        sl = (slice(y0, y0 + ch), slice(x0, x0 + cw))
        return img1[sl], img2[sl], flow[sl]

    def __call__(self, img1, img2, flow):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow = self.spatial_transform(img1, img2, flow)
        return (np.ascontiguousarray(img1), np.ascontiguousarray(img2),
                np.ascontiguousarray(flow, dtype=np.float32))


class SparseFlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=False):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.3, contrast=0.3, saturation=0.3, hue=0.3 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        stack = self.photo_aug(np.concatenate([img1, img2], axis=0))
        return tuple(np.split(stack, 2, axis=0))

    def eraser_transform(self, img1, img2):
        return _erase(img1, img2, self.eraser_aug_prob)

    def resize_sparse_flow_map(self, flow, valid, fx=1.0, fy=1.0):
        return sparse_flow_resize(flow, valid, fx, fy)

    def spatial_transform(self, img1, img2, flow, valid):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 1) / float(ht),
                               (self.crop_size[1] + 1) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = float(np.clip(scale, min_scale, None))
        scale_y = float(np.clip(scale, min_scale, None))
        if np.random.rand() < self.spatial_aug_prob:
            img1 = _resize(img1, scale_x, scale_y)
            img2 = _resize(img2, scale_x, scale_y)
            flow, valid = self.resize_sparse_flow_map(flow, valid, fx=scale_x, fy=scale_y)
        if self.do_flip and np.random.rand() < 0.5:
            img1, img2 = img1[:, ::-1], img2[:, ::-1]
            flow = flow[:, ::-1] * np.array([-1.0, 1.0], np.float32)
            valid = valid[:, ::-1]
        margin_y, margin_x = 20, 50
        y0 = np.random.randint(0, img1.shape[0] - self.crop_size[0] + margin_y)
        x0 = np.random.randint(-margin_x, img1.shape[1] - self.crop_size[1] + margin_x)
        y0 = int(np.clip(y0, 0, img1.shape[0] - self.crop_size[0]))
        x0 = int(np.clip(x0, 0, img1.shape[1] - self.crop_size[1]))
        sl = (slice(y0, y0 + self.crop_size[0]), slice(x0, x0 + self.crop_size[1]))
        return img1[sl], img2[sl], flow[sl], valid[sl]

    def __call__(self, img1, img2, flow, valid):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow, valid = self.spatial_transform(img1, img2, flow, valid)
        return (np.ascontiguousarray(img1), np.ascontiguousarray(img2),
                np.ascontiguousarray(flow, dtype=np.float32), np.ascontiguousarray(valid))
