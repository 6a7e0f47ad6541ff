"""Fused inference engine for the RAFT refinement loop (bf16, MI355X).

Replaces, for inference (no autograd, bf16 autocast), the per-iteration
module graph of reference core/raft.py:122-139 + core/update.py (motion
encoder, ConvGRU / SepConvGRU, flow head, mask head, ~40 kernels and
several concatenations per iteration) with a fixed sequence of hand-written
HIP launches over persistent channels-last buffers:

  full RAFT, per iteration (12 launches, +2 on iterations that upsample):
    corr_lookup_into   pyramid window lookup -> corr[., 384]   (324 + zero pad)
    flow_encode        convf1 7x7 of (coords1 - grid), ReLU   -> f1[., 128];
                       flow (bf16) -> hx[., 382:384]
    conv convc1 1x1    corr -> c1 (ReLU)
    conv convc2 3x3    c1 -> mot[., 0:192] (ReLU)
    conv convf2 3x3    f1 -> mot[., 192:256] (ReLU)
    conv conv   3x3    mot -> hx[., 256:382] (ReLU)          (= cat[out, flow])
    conv z|r 1x5       hx -> z, r*h          (GRU gate epilogue)
    conv q   1x5       [r*h | hx[128:]] -> hx[., 0:128] = (1-z)h + z tanh(q)
    conv z|r, q 5x1    (second SepConvGRU pass)
    conv head 3x3      h -> [flow-head hidden | mask hidden] (ReLU; one GEMM,
                       the mask half only on iterations that upsample)
    flow_head 3x3      -> coords1 += delta   (VALU kernel, csrc/flowhead.hip)
    conv mask 1x1      -> mask x 0.25        (upsampling iterations only)
    convex_upsample    (upsampling iterations only)

  hx = [h | inp | motion | flow] is ONE buffer, so cat[h, x] and
  cat[r*h, x] are just different segment views of it.

RAFT-small uses the same machinery (ConvGRU 3x3, hidden 96, context 64,
corr radius 3 -> 196 channels, bilinear x8 upsampling).

Packed weights are cached per (parameter versions) and rebuilt after any
in-place update, so an optimizer step between evaluations is picked up.

fp32 (the reference's default inference precision, evaluate.py:174 /
rafttoonnx.py): the same sequence on fp32 buffers, every conv on the
split-bf16 F32 tiles (csrc/conv.hip conv_lds_kernel<..., F32>: x.w as three
bf16 MFMA products, ~2^-17 relative error), the flow encoder / flow head /
lookup / upsampling in their fp32 forms.
"""
from __future__ import annotations


import os

import torch
import torch.nn.functional as F

from ..ops import _ext
from ..ops.conv import (EPI_FLOW, EPI_GRU_Q, EPI_GRU_ZR, EPI_RELU, EPI_SCALE, choose_tile_f32, conv_fused,
                        frag32_eligible, frag_eligible, frag_weight, frag_weight_split, pack_bias, pack_weight,
                        pack_weight_split, pad_to)

_F32_ENGINE = True
# RAFT-small inference: the flow branch on the side stream as well (RS_SMALL_SIDE=0 to
# compare; 1.914-1.941 -> 1.848-1.900 ms per 1088x436 pair, profiles/r6/ab_small_side_s30.txt)
_SMALL_SIDE = os.environ.get("RS_SMALL_SIDE", "1") == "1"
from ..ops.upsample import convex_upsample


# RAFT-small head conv K in bf16 (96 channels padded to 128 with zero weights:
# K % 64, so the weight-streaming tiles can serve it; profiles/r5/README.md)
_SMALL_HEAD_K = 128
# ... and its GRU-q conv's input segments padded to 64-multiples (bf16)
_SMALL_Q_PAD = True


class _Conv:
    """One packed convolution: weight [Cout_pad][taps][Ktot] bf16 + fp32 bias."""

    def __init__(self, convs, segs, f32=False):
        convs = convs if isinstance(convs, (list, tuple)) else [convs]
        weight = torch.cat([c.weight for c in convs], 0)
        bias = torch.cat([c.bias for c in convs], 0)
        self.cout = weight.shape[0]
        self.kh, self.kw = weight.shape[2], weight.shape[3]
        pack = pack_weight_split if f32 else pack_weight
        self.w = pack(weight, segs, pad_to(self.cout, 128))
        self.b = pack_bias(bias)
        # fragment-major copy for the weight-streaming tiles (bf16 3x3 / 1x5 / 5x1 only;
        # fp32: the split [frag(wh); frag(wl)] of tiles 81-83, on the split weight's _rs_frag32)
        self.wf = frag_weight(self.w) if not f32 and frag_eligible(self.w, self.kh, self.kw) else None
        if f32 and frag32_eligible(self.w, self.kh, self.kw):
            self.w._rs_frag32 = frag_weight_split(self.w)


def _copy_conv(prev: "_Conv", new: "_Conv"):
    prev.w.copy_(new.w)
    f_prev, f_new = getattr(prev.w, "_rs_frag32", None), getattr(new.w, "_rs_frag32", None)
    if f_prev is not None and f_new is not None:
        f_prev.copy_(f_new)
    prev.b.copy_(new.b)
    if prev.wf is not None and new.wf is not None:
        prev.wf.copy_(new.wf)
    else:
        prev.wf = new.wf


class FusedUpdate:
    def __init__(self, model):
        self.model = model
        self.key = None
        self.bufs = {}

    # ------------------------------------------------------------ eligibility
    @staticmethod
    def eligible(model, image, corr_fn) -> bool:
        if image.device.type != "cuda" or torch.is_grad_enabled():
            return False
        if not model.cfg.fused_gru or not (model.cfg.mixed_precision or _F32_ENGINE):
            return False
        if not _ext.use_hip(image):
            return False
        return getattr(corr_fn, "hip", False)  # all-pairs pyramid or on-the-fly (HIP) correlation

    # ------------------------------------------------------------ weights
    def _version_key(self):
        from ..runtime.weights import generation
        return ((generation(), bool(self.model.cfg.mixed_precision))
                + tuple((p.data_ptr(), p._version) for p in self.model.update_block.parameters()))

    @torch.no_grad()
    def _pack(self):
        ub = self.model.update_block
        small = self.model.cfg.small
        self.f32 = f32 = not self.model.cfg.mixed_precision
        _C = lambda convs, segs: _Conv(convs, segs, f32)  # noqa: E731
        if small:
            hd, cd, corr_c = 96, 64, 4 * 49
            self.corr_pad = pad_to(corr_c, 64)   # 256 (64-deep K steps)
            enc = ub.encoder
            # hx = [h 96 | inp 64 | mot 80 | flow 2 | pad 14] = 256
            self.hx_c, self.off_inp, self.off_mot, self.off_flow = 256, 96, 160, 240
            self.mot_c = 128                    # [c1 96 | f2 32]
            self.convc1 = _C(enc.convc1, [(self.corr_pad, [(0, corr_c, 0)])])
            self.convf2 = _C(enc.convf2, [(64, [(0, 64, 0)])])
            self.conv = _C(enc.conv, [(128, [(0, 128, 0)])])
            self.f1_c = 64
            gru = ub.gru
            if f32 or not _SMALL_Q_PAD:
                q_segs = [(pad_to(hd, 32), [(0, hd, 0)]), (160, [(hd, cd + 82, 0)])]
                self.rh_c, self.q_xoff = pad_to(hd, 32), hd
            else:
                # bf16: segments of 64-multiples for the 64-deep-K tiles -- r*h in a
                # 128-channel buffer (channels 96.. stay zero) and x read as
                # hx[64:256] (h[64:96] and the pad meet zero weights)
                q_segs = [(128, [(0, hd, 0)]), (192, [(hd, cd + 82, hd - 64)])]
                self.rh_c, self.q_xoff = 128, 64
            self.gru = [(
                _C([gru.convz, gru.convr], [(256, [(0, hd, 0), (hd, cd + 82, hd)])]),
                _C(gru.convq, q_segs),
            )]
            # bf16: K padded to 128 (hx[96:128] meets zero weights) so the
            # weight-streaming tiles (K % 64) can serve it on batch-1 grids
            self.head_k = 96 if f32 else _SMALL_HEAD_K
            self.head = _C(ub.flow_head.conv1, [(self.head_k, [(0, hd, 0)])])
            self.head_c = 128
            self.flow = _C(ub.flow_head.conv2, [(128, [(0, 128, 0)])])
            self.mask0 = self.mask2 = None
        else:
            hd, cd, corr_c = 128, 128, 4 * 81
            self.corr_pad = pad_to(corr_c, 64)   # 384 (64-deep K steps)
            enc = ub.encoder
            # hx = [h 128 | inp 128 | mot 126 | flow 2] = 384
            self.hx_c, self.off_inp, self.off_mot, self.off_flow = 384, 128, 256, 382
            self.mot_c = 256                    # [c2 192 | f2 64]
            self.convc1 = _C(enc.convc1, [(self.corr_pad, [(0, corr_c, 0)])])
            self.convc2 = _C(enc.convc2, [(256, [(0, 256, 0)])])
            self.convf2 = _C(enc.convf2, [(128, [(0, 128, 0)])])
            self.conv = _C(enc.conv, [(256, [(0, 256, 0)])])
            self.f1_c = 128
            g = ub.gru
            self.gru = []
            for zc, rc, qc in ((g.convz1, g.convr1, g.convq1), (g.convz2, g.convr2, g.convq2)):
                self.gru.append((
                    _C([zc, rc], [(384, [(0, 384, 0)])]),
                    _C(qc, [(128, [(0, hd, 0)]), (256, [(hd, 256, 0)])]),
                ))
            self.head = _C([ub.flow_head.conv1, ub.mask[0]], [(128, [(0, hd, 0)])])
            self.head_c = 512
            self.flow = _C(ub.flow_head.conv2, [(256, [(0, 256, 0)])])
            self.mask2 = _C(ub.mask[2], [(256, [(0, 256, 0)])])
        self.hd, self.cd = hd, cd
        if not small:
            self.rh_c, self.q_xoff = pad_to(hd, 32), hd
        f1 = ub.encoder.convf1
        self.f1_w = f1.weight.detach().float().permute(2, 3, 1, 0).contiguous()  # [7][7][2][Cout]
        self.f1_b = f1.bias.detach().float().contiguous()
        fc = ub.flow_head.conv2  # 2-channel output conv: VALU kernel (csrc/flowhead.hip)
        self.flow_w32 = fc.weight.detach().float().permute(0, 2, 3, 1).contiguous()  # [2][3][3][Cin]
        self.flow_b32 = fc.bias.detach().float().contiguous()

    def _reuse_storage(self, old):
        """Copy freshly packed weights into the previous tensors (same shapes),
        so hipGraphs captured against them stay valid after a weight update."""
        for name, new in list(self.__dict__.items()):
            prev = old.get(name)
            if isinstance(new, _Conv) and isinstance(prev, _Conv) and prev.w.shape == new.w.shape:
                _copy_conv(prev, new)
                self.__dict__[name] = prev
            elif name == "gru" and isinstance(prev, list) and len(prev) == len(new):
                for (pz, pq), (nz, nq) in zip(prev, new):
                    for p_, n_ in ((pz, nz), (pq, nq)):
                        _copy_conv(p_, n_)
                self.gru = prev
            elif name in ("f1_w", "f1_b", "flow_w32", "flow_b32") and isinstance(prev, torch.Tensor) and prev.shape == new.shape:
                prev.copy_(new)
                self.__dict__[name] = prev

    def _buffers(self, B, H, W, dev):
        key = (B, H, W, dev, self.f32)
        bufs = self.bufs.get(key)
        if bufs is None:
            dt = torch.float32 if self.f32 else torch.bfloat16
            e = lambda c: torch.empty(B, H, W, c, device=dev, dtype=dt)  # noqa: E731
            z = lambda c: torch.zeros(B, H, W, c, device=dev, dtype=dt)  # noqa: E731
            bufs = dict(corr=z(self.corr_pad), f1=e(self.f1_c), mot=e(self.mot_c), hx=z(self.hx_c),
                        z=e(self.hd), rh=z(self.rh_c), head=e(self.head_c))
            if not self.model.cfg.small:
                bufs["c1"] = e(256)
                bufs["mask"] = e(576)
            # kept for every shape seen: a captured hipGraph references them
            self.bufs[key] = bufs
        return bufs

    # ------------------------------------------------------------ run
    @torch.no_grad()
    def refresh(self):
        """Re-pack after a weight update, into the existing storage."""
        k = self._version_key()
        if k != self.key:
            old = self.__dict__.copy()
            self._pack()
            self._reuse_storage(old)
            self.key = k

    @torch.no_grad()
    def run(self, net, inp, corr_fn, coords0, coords1, iters, test_mode):
        """inp None: ``net`` is the context encoder's raw (hd + cd)-channel output."""
        self.refresh()
        B, _, H, W = coords1.shape
        bufs = self._buffers(B, H, W, coords1.device)
        hx = bufs["hx"]
        hd = self.hd
        if self.f32:  # split-bf16 F32 tiles (fp32 activations)
            P = B * H * W

            def cf(segs, w, b, kh, kw, cout, epi, out, ooff=0, **kw_):
                conv_fused(segs, w, b, kh, kw, cout, epi, out, ooff, tile=None, **kw_)  # tuned F32 table / heuristic
        else:
            cf = conv_fused
        if inp is None:
            # net: the context encoder's raw output -- split + tanh / relu
            # (reference core/raft.py:108-110) straight into the hx slots, one pass
            cn = net.permute(0, 2, 3, 1).to(hx.dtype).contiguous()
            torch.ops.raft_stir.context_act(cn, hx, hx[..., self.off_inp:self.off_inp + self.cd], hd)
        else:
            hx[..., :hd].copy_(net.permute(0, 2, 3, 1))
            hx[..., self.off_inp:self.off_inp + self.cd].copy_(inp.permute(0, 2, 3, 1))
        coords1 = coords1.float().contiguous().clone()
        st = getattr(corr_fn, "state", None)  # None: on-the-fly correlation
        small = self.model.cfg.small
        preds, flow_up = [], None
        # flow branch (flow encoder + convf2) on the second HIP stream, parallel
        # to the correlation branch (lookup + convc1 + convc2): at batch 1 each
        # of these convs fills only part of the 256 CUs.  Both write disjoint
        # channel ranges of `mot`; joined before the conv that reads it.
        main = torch.cuda.current_stream(coords1.device)
        side = (self.model._side_stream(coords1.device)
                if ((not small or _SMALL_SIDE) and self.model.cfg.overlap_encoders) else None)
        for itr in range(iters):
            want_up = (not test_mode) or itr == iters - 1
            if side is not None:
                side.wait_stream(main)  # coords1 of the previous iteration
                with torch.cuda.stream(side):
                    torch.ops.raft_stir.flow_encode(coords1, self.f1_w, self.f1_b, bufs["f1"], 0, hx, self.off_flow)
                    if small:
                        cf([(bufs["f1"], 0, 64)], self.convf2.w, self.convf2.b, 3, 3, 32, EPI_RELU,
                           bufs["mot"], 96, wf=self.convf2.wf)
                    else:
                        cf([(bufs["f1"], 0, 128)], self.convf2.w, self.convf2.b, 3, 3, 64, EPI_RELU,
                           bufs["mot"], 192, wf=self.convf2.wf)
            if st is not None:
                torch.ops.raft_stir.corr_lookup_into(st.pyr, coords1, st.radius, bufs["corr"])
            else:  # memory-efficient path: correlate the pooled fmap2 pyramid on the fly
                c = torch.ops.raft_stir.corr_otf(corr_fn.f1, corr_fn.f2s, coords1, corr_fn.radius, corr_fn.scale,
                                                 not self.f32)
                bufs["corr"][..., :c.shape[-1]].copy_(c)
            if side is None:
                torch.ops.raft_stir.flow_encode(coords1, self.f1_w, self.f1_b, bufs["f1"], 0, hx, self.off_flow)
            cp = self.corr_pad
            if small:
                cf([(bufs["corr"], 0, cp)], self.convc1.w, self.convc1.b, 1, 1, 96, EPI_RELU,
                           bufs["mot"], 0)
                if side is None:
                    cf([(bufs["f1"], 0, 64)], self.convf2.w, self.convf2.b, 3, 3, 32, EPI_RELU,
                       bufs["mot"], 96, wf=self.convf2.wf)
                else:
                    main.wait_stream(side)
                cf([(bufs["mot"], 0, 128)], self.conv.w, self.conv.b, 3, 3, 80, EPI_RELU,
                           hx, self.off_mot, wf=self.conv.wf)
            else:
                cf([(bufs["corr"], 0, cp)], self.convc1.w, self.convc1.b, 1, 1, 256, EPI_RELU,
                           bufs["c1"], 0)
                cf([(bufs["c1"], 0, 256)], self.convc2.w, self.convc2.b, 3, 3, 192, EPI_RELU,
                           bufs["mot"], 0, wf=self.convc2.wf)
                if side is None:
                    cf([(bufs["f1"], 0, 128)], self.convf2.w, self.convf2.b, 3, 3, 64, EPI_RELU,
                               bufs["mot"], 192, wf=self.convf2.wf)
                else:
                    main.wait_stream(side)
                cf([(bufs["mot"], 0, 256)], self.conv.w, self.conv.b, 3, 3, 126, EPI_RELU,
                           hx, self.off_mot, wf=self.conv.wf)
            for zr, q in self.gru:
                rhc = bufs["rh"].shape[-1]
                cf([(hx, 0, self.hx_c)], zr.w, zr.b, zr.kh, zr.kw, 2 * hd, EPI_GRU_ZR,
                           bufs["z"], 0, hd=hd, out2=bufs["rh"], o2off=0, aux1=hx, a1off=0, wf=zr.wf)
                cf([(bufs["rh"], 0, rhc), (hx, self.q_xoff, self.hx_c - self.q_xoff)], q.w, q.b, q.kh, q.kw, hd,
                           EPI_GRU_Q, hx, 0, aux1=hx, a1off=0, aux2=bufs["z"], a2off=0, wf=q.wf)
            if small:
                cf([(hx, 0, self.head_k)], self.head.w, self.head.b, 3, 3, 128, EPI_RELU, bufs["head"], 0,
                   wf=self.head.wf)
                torch.ops.raft_stir.flow_head(bufs["head"], 0, 128, self.flow_w32, self.flow_b32, coords1, None)
            else:
                cf([(hx, 0, hd)], self.head.w, self.head.b, 3, 3, 512 if want_up else 256, EPI_RELU,
                           bufs["head"], 0, wf=self.head.wf)
                torch.ops.raft_stir.flow_head(bufs["head"], 0, 256, self.flow_w32, self.flow_b32, coords1, None)
            if not want_up:
                continue
            flow = coords1 - coords0
            if small:
                flow_up = 8 * F.interpolate(flow, size=(8 * H, 8 * W), mode="bilinear", align_corners=True)
            else:
                cf([(bufs["head"], 256, 256)], self.mask2.w, self.mask2.b, 1, 1, 576, EPI_SCALE,
                           bufs["mask"], 0, scale=0.25)
                flow_up = convex_upsample(flow, bufs["mask"].permute(0, 3, 1, 2))
            preds.append(flow_up)
        return coords1, preds, flow_up
