"""InputPadder: replicate-pad to a multiple of 8 and unpad (reference core/utils/utils.py:7-24).

mode 'sintel' splits the padding between both sides; any other mode ('kitti')
pads the bottom (and splits the width).
"""
from __future__ import annotations

import torch.nn.functional as F


class InputPadder:
    def __init__(self, dims, mode="sintel", multiple=8):
        self.ht, self.wd = dims[-2:]
        ph = (-self.ht) % multiple
        pw = (-self.wd) % multiple
        left, right = pw // 2, pw - pw // 2
        if mode == "sintel":
            self._pad = [left, right, ph // 2, ph - ph // 2]
        else:
            self._pad = [left, right, 0, ph]

    def pad(self, *inputs):
        return [F.pad(x, self._pad, mode="replicate") for x in inputs]

    def unpad(self, x):
        ht, wd = x.shape[-2:]
        t, b, l, r = self._pad[2], ht - self._pad[3], self._pad[0], wd - self._pad[1]
        return x[..., t:b, l:r]
