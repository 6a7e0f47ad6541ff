"""Fused TRAINING engine for the RAFT refinement loop (RAFT and RAFT-small; bf16
under --mixed_precision, fp32 otherwise -- the reference's standard schedule,
/root/reference/train_standard.sh:3-6).

One ``torch.autograd.Function`` covers the whole 12-iteration refinement
loop of reference core/raft.py:122-139 (update block of core/update.py).

Forward: the same hand-written HIP launches as the inference engine
(models/fused_update.py), but every activation a gradient needs is written
into an [iters * B, H, W, C] slot instead of being overwritten:

  S.corr, S.c1, S.f1, S.mot  motion-encoder inputs / ReLU outputs
  S.hx[i] = [h_i | motion_i (126) | flow_i (2)]   (iters + 1 slots: h after pass 2)
  S.h1                        h after the first SepConvGRU pass
  S.z / S.r / S.q / S.rh      GRU gates, tanh(q), r*h per pass
  S.head, S.mask              flow-head/mask hidden (ReLU), convex mask
  S.C[i]                      coords before update i (iters + 1 slots)

The convex upsampling of all iterations is one launch after the loop (the
predictions do not feed back), so the Function returns one
[iters * B, 2, 8H, 8W] tensor that the model splits into views; the fused
sequence loss (train/loss.py) consumes it whole.

Weights are packed for the kernels by one static gather per step (and the
gradients unpacked by one), see FusedTrainEngine._build_maps.

Backward: one batched convex_upsample_backward, then iteration by iteration
in reverse (dgrads = the forward conv kernel with transposed + flipped
packed weights and gradient epilogues):

  mask2 / flow dgrad (through the hidden ReLU)  -> d head
  head dgrad             -> dh  (fp32, accumulated with dh of iteration i+1)
  GRU pass 2, pass 1     -> gate backward kernel, q-conv dgrad with the
                            r-gate epilogue, zr-conv dgrad (fp32 accumulation
                            into G = [dh | d inp | d motion])
  motion encoder dgrads  -> d corr -> pyramid window-lookup backward
                            (into the CorrState pyramid gradient; the volume
                            node folds it into d fmap1 / d fmap2 afterwards)

Every conv's weight gradient is then ONE batched MFMA GEMM over all
iterations' pixels (csrc/conv_wgrad.hip) instead of 12 per-iteration GEMMs
and 12 accumulations, and every bias gradient one column sum.

Numerics: bf16 operands, fp32 accumulation everywhere, fp32 gradient
accumulators for the recurrent state -- the same contract as the reference's
autocast training (which used fp16).

fp32 (``cfg.mixed_precision`` off): every activation / gradient slot is fp32;
the convolutions (forward and dgrad) run on the split-bf16 F32 tiles of
csrc/conv.hip (x = xh + xl, w = wh + wl, x.w ~= xh.wh + xl.wh + xh.wl: relative
error ~2^-17) with the packed weights in their [wh | wl] layout, and each
weight gradient is the same bf16 MFMA GEMM run on the three split products
(dYh.Xh + dYl.Xh + dYh.Xl, bias gradient from dYh + dYl).  The gate, ReLU,
flow-head, flow-encoder, lookup and upsampling kernels run their fp32
instantiations.
"""
from __future__ import annotations

import contextlib
import os


import torch

from ..ops import _ext
from ..ops.conv import (EPI_ACC_F32, EPI_BIAS, EPI_FLOW, EPI_GRU_Q, EPI_GRU_QBWD, EPI_GRU_ZR, EPI_RELU,
                        EPI_RELU_BWD, EPI_SCALE, conv_fused, frag32_eligible, frag_eligible, frag_weight,
                        frag_weight_split, pack_bias, pack_weight, pad_to)

R = torch.ops.raft_stir
HD = 128          # hidden dim (full RAFT)
CORR_C = 324
CORR_PAD = 384
SHD = 96          # RAFT-small: hidden dim, 4 levels x 7 x 7 correlation taps (radius 3)
SCORR_C = 196
SCORR_PAD = 256
# RAFT-small bf16: the GRU-q and head forward and the q / conv / convc1 dgrads
# read 64-multiple K windows (zero weights on the padding) so that the
# weight-streaming tiles (3x3) and the 1x1 GEMM serve them instead of the
# 32-deep-K register tiles (inference does the same, models/fused_update.py)
_SMALL_KPAD = os.environ.get("RS_SMALL_KPAD", "1") != "0"
# the all-pairs volume backward issued by the engine right after the last
# lookup backward, ahead of the weight-gradient issue (ops/corr.py
# CorrState.early_backward); RS_EARLY_CORR_BWD=0 leaves it to autograd
_EARLY_CORR_BWD = os.environ.get("RS_EARLY_CORR_BWD", "1") != "0"
# fp32 engine: split fragment-major copies of the packed weights for the fp32
# weight-streaming tiles (csrc/conv_v3f.hip), made per step after the gather
_V3F_TRAIN = True


class _PConv:
    """A conv of the update block: forward packing, dgrad packing, grad unpacking."""

    def __init__(self, convs, segs, scale=1.0, wsegs=None, fsegs=None, dk=None):
        self.convs = convs if isinstance(convs, (list, tuple)) else [convs]
        self.segs = segs          # [(C, [(w0, n, s0), ...]), ...] as in pack_weight
        # the forward's own input windows (default: segs, which also define the
        # dgrad's output channels) and the dgrad's K (default: Cout to 32)
        self.fsegs = fsegs if fsegs is not None else segs
        self.dk = dk
        # segment layout of the weight-gradient GEMM (its K segments must be
        # multiples of 64: RAFT-small reads wider, zero-weighted windows there)
        self.wsegs = wsegs if wsegs is not None else segs
        self.scale = scale        # output scale folded into the epilogue (mask x 0.25)
        w0 = self.convs[0].weight
        self.kh, self.kw = w0.shape[2], w0.shape[3]
        self.cout = sum(c.weight.shape[0] for c in self.convs)
        self.cin = w0.shape[1]
        self.ktot = sum(c for c, _ in segs)
        self.wktot = sum(c for c, _ in self.wsegs)

    def index_maps(self, pidx, fill, frag=False):
        """Index maps (into the flat parameter vector) of the packed forward
        weight [Cout_pad128][taps][Ktot], the bias, and the dgrad weight
        Wd[k][tap'][co] = W[co][taps-1-tap'][k] ([pad128(Ktot)][taps][pad32(Cout)]);
        with ``frag`` also the fragment-major copies of both (ops/conv.py
        frag_weight; None where the weight-streaming tiles cannot serve them)."""
        weight = torch.cat([pidx[id(c.weight)] for c in self.convs], 0)
        bias = torch.cat([pidx[id(c.bias)] for c in self.convs], 0)
        cout, cin, kh, kw = weight.shape
        taps = kh * kw
        wt = weight.permute(0, 2, 3, 1).reshape(cout, taps, cin)

        def packed(segs):
            w = torch.full((pad_to(cout, 128), taps, sum(c for c, _ in segs)), fill, dtype=torch.long)
            kb = 0
            for c, pieces in segs:
                for w0, n, s0 in pieces:
                    w[:cout, :, kb + s0:kb + s0 + n] = wt[:, :, w0:w0 + n]
                kb += c
            return w
        ws = packed(self.segs)
        w = ws if self.fsegs is self.segs else packed(self.fsegs)
        # the dgrad's K = the gradient slot width (32-channel granules, or dk)
        cy = self.dk or pad_to(cout, 32)
        wd = torch.full((pad_to(self.ktot, 128), taps, cy), fill, dtype=torch.long)
        wd[:self.ktot] = ws[:cy].flip(1).permute(2, 1, 0)
        self.cy = cy
        wf = frag_weight(w) if frag and frag_eligible(w, kh, kw) else None
        wdf = frag_weight(wd) if frag and frag_eligible(wd, kh, kw) else None
        return w, bias, wd, wf, wdf

    def grad_maps(self, gidx):
        """Per original conv (weight, bias) index maps into the packed gradient
        buffers gidx = (dW [Cout_pad128][taps][Ktot], db [Cout]) index views."""
        dwi, dbi = gidx
        taps = self.kh * self.kw
        gw = torch.empty(self.cout, taps, self.cin, dtype=torch.long)
        kb = 0
        for c, pieces in self.wsegs:
            for w0, n, s0 in pieces:
                gw[:, :, w0:w0 + n] = dwi[:self.cout, :, kb + s0:kb + s0 + n]
            kb += c
        gw = gw.reshape(self.cout, self.kh, self.kw, self.cin).permute(0, 3, 1, 2)
        out, r0 = [], 0
        for c in self.convs:
            n = c.weight.shape[0]
            out.append((gw[r0:r0 + n].contiguous(), dbi[r0:r0 + n].contiguous()))
            r0 += n
        return out


class FusedTrainEngine:
    def __init__(self, model):
        self.model = model
        ub = model.update_block
        enc, g = ub.encoder, ub.gru
        full = lambda c: [(c, [(0, c, 0)])]
        self.small = bool(model.cfg.small)
        # fp32 training (the reference's default precision): fp32 slots, split-bf16 kernels
        self.f32 = not bool(model.cfg.mixed_precision)
        self.spad = self.small and not self.f32 and _SMALL_KPAD
        if self.small:
            # RAFT-small (reference core/update.py SmallMotionEncoder / ConvGRU /
            # FlowHead(96, 128)): hx slot = [h 96 | inp 64 | motion 80 | flow 2 | 0 14]
            # = cat[h, x] of the ConvGRU in ONE 256-channel window
            self.hd, self.hx_c, self.corr_c, self.corr_pad = SHD, 256, SCORR_C, SCORR_PAD
            dk = 128 if self.spad else None
            self.c1 = _PConv(enc.convc1, [(SCORR_PAD, [(0, SCORR_C, 0)])], dk=dk)
            self.f2 = _PConv(enc.convf2, full(64))
            self.cv = _PConv(enc.conv, full(128), dk=dk)
            self.zr = [_PConv([g.convz, g.convr], [(256, [(0, SHD + 146, 0)])])]
            # q reads [r*h | x]; its weight gradient (and the padded bf16
            # forward) reads 64-aligned windows (r*h slot zero-padded to 128,
            # x from hx[64:256] with zero weights on h[64:96])
            qw = [(128, [(0, SHD, 0)]), (192, [(SHD, 146, 32)])]
            self.q = [_PConv(g.convq, [(SHD, [(0, SHD, 0)]), (160, [(SHD, 146, 0)])], wsegs=qw,
                             fsegs=qw if self.spad else None, dk=dk)]
            hw = [(128, [(0, SHD, 0)])]  # h' with inp[0:32] behind it (zero weights)
            self.head = _PConv(ub.flow_head.conv1, full(SHD), wsegs=hw, fsegs=hw if self.spad else None)
            self.flow = _PConv(ub.flow_head.conv2, full(128))
            self.mask2 = None
            self.c2 = None
            self.convs = [self.c1, self.f2, self.cv, *self.zr, *self.q, self.head, self.flow]
        else:
            self.hd, self.hx_c, self.corr_c, self.corr_pad = HD, 256, CORR_C, CORR_PAD
            gru_segs = [(HD, [(0, HD, 0)]), (128, [(HD, 128, 0)]), (128, [(HD + 128, 128, 0)])]
            self.c1 = _PConv(enc.convc1, [(CORR_PAD, [(0, CORR_C, 0)])])
            self.c2 = _PConv(enc.convc2, full(256))
            self.f2 = _PConv(enc.convf2, full(128))
            self.cv = _PConv(enc.conv, full(256))
            self.zr = [_PConv([g.convz1, g.convr1], gru_segs), _PConv([g.convz2, g.convr2], gru_segs)]
            self.q = [_PConv(g.convq1, gru_segs), _PConv(g.convq2, gru_segs)]
            self.head = _PConv([ub.flow_head.conv1, ub.mask[0]], full(HD))
            self.flow = _PConv(ub.flow_head.conv2, full(256))
            self.mask2 = _PConv(ub.mask[2], full(256), scale=0.25)
            self.convs = [self.c1, self.c2, self.f2, self.cv, *self.zr, *self.q, self.head, self.flow, self.mask2]
        self.f1 = enc.convf1
        self.f1c = self.f1.weight.shape[0]
        self.adt = torch.float32 if self.f32 else torch.bfloat16
        # parameter order handed to autograd (grads are returned in this order)
        self.params = []
        for pc in self.convs:
            for c in pc.convs:
                self.params += [c.weight, c.bias]
        self.params += [self.f1.weight, self.f1.bias]
        self._bufs = {}
        self._maps = None
        self.grad_group = None     # (process group, world size): packed gradient all-reduce
        self.trace = None          # optional list: ("packed_allreduce", ...) events (tests)

    def attach_grad_group(self, group, world_size: int):
        """Data parallelism: all-reduce (average) the packed update-block
        gradient buffer over ``group`` from the weight-gradient stream, as one
        collective overlapping the encoder backward (parallel/dist.py)."""
        self.grad_group = (group, int(world_size))

    def reduce_packed(self, gbuf):
        """Average ``gbuf`` over the attached group.  Issued on the CURRENT
        stream (the weight-gradient stream when deferred): the process group's
        RCCL stream waits for it, and ``work.wait()`` makes the current stream
        -- not the host, not the main stream -- wait for the collective."""
        import torch.distributed as dist
        group, ws = self.grad_group
        if ws > 1:
            gbuf.mul_(1.0 / ws)
        work = dist.all_reduce(gbuf, group=group, async_op=True)
        if self.trace is not None:
            self.trace.append(("packed_allreduce", gbuf.numel()))
        work.wait()

    def _build_maps(self, dev):
        """Static gather maps: packing every update-block weight for the fused
        kernels (forward + dgrad layouts) is ONE index_select over the
        concatenated parameters per step, and unpacking every weight / bias
        gradient from the kernels' packed accumulators ONE index_select over
        the flat gradient buffer -- instead of ~200 small copy kernels."""
        sizes = [p.numel() for p in self.params]
        nsrc = sum(sizes)
        fill = nsrc  # index of the appended zero
        ids = torch.arange(nsrc)
        pidx, off = {}, 0
        for p in self.params:
            pidx[id(p)] = ids[off:off + p.numel()].view(p.shape)
            off += p.numel()
        bf_maps, f32_maps, layout = [], [], []
        nbf = 0
        for pc in self.convs:
            w, b, wd, wf, wdf = pc.index_maps(pidx, fill, frag=not self.f32)
            layout.append((pc, w.shape, wd.shape, b.shape, wf is not None, wdf is not None))
            bf_maps += [w.reshape(-1), wd.reshape(-1)]
            bf_maps += [x.reshape(-1) for x in (wf, wdf) if x is not None]
            f32_maps.append(b.reshape(-1))
        f1w = pidx[id(self.f1.weight)].permute(2, 3, 1, 0).contiguous()  # [7][7][2][f1c]
        f32_maps += [f1w.reshape(-1), pidx[id(self.f1.bias)].reshape(-1)]
        # the 2-channel flow output conv in csrc/flowhead.hip's fp32 [2][3][3][Cin] layout
        fcw = self.model.update_block.flow_head.conv2.weight
        f32_maps.append(pidx[id(fcw)].permute(0, 2, 3, 1).reshape(-1))
        nbf = sum(m.numel() for m in bf_maps)
        gather = torch.cat(bf_maps + f32_maps)
        # scale (mask x 0.25) folded into the dgrad weights: element range in the bf16 region
        o, scaled = 0, []
        for pc, ws, wds, bs, hf, hdf in layout:
            o += ws.numel()
            if pc.scale != 1.0:
                scaled.append((o, o + wds.numel(), pc.scale))
            o += wds.numel()
            o += ws.numel() if hf else 0
            if hdf and pc.scale != 1.0:
                scaled.append((o, o + wds.numel(), pc.scale))
            o += wds.numel() if hdf else 0
        # gradient buffer: per conv dW [Cout_pad128][taps][Ktot] + db [Cout], then flow-conv dW, db
        glayout, go = [], 0
        for pc in self.convs:
            dws = (pad_to(pc.cout, 128), pc.kh * pc.kw, pc.wktot)
            n = dws[0] * dws[1] * dws[2]
            glayout.append((go, dws, go + n, pc.cout))
            go += n + pc.cout
        fc = self.f1c
        gf1 = (go, go + 49 * 2 * fc)
        gtotal = gf1[1] + fc
        gids = torch.arange(gtotal)
        gmaps, gscaled, o = [], [], 0
        for pc, (dwo, dws, dbo, nb) in zip(self.convs, glayout):
            dwi = gids[dwo:dwo + dws[0] * dws[1] * dws[2]].view(dws)
            dbi = gids[dbo:dbo + nb]
            for gw, gb in pc.grad_maps((dwi, dbi)):
                gmaps += [gw.reshape(-1), gb.reshape(-1)]
                if pc.scale != 1.0:
                    scaled_range = (o, o + gw.numel() + gb.numel(), pc.scale)
                    gscaled.append(scaled_range)
                o += gw.numel() + gb.numel()
        f1g = gids[gf1[0]:gf1[1]].view(7, 7, 2, fc).permute(3, 2, 0, 1).contiguous()
        gmaps += [f1g.reshape(-1), gids[gf1[1]:gf1[1] + fc]]
        # the same gather as per-element codes (source param << 24 | index) for
        # csrc/wpack.hip: one launch per dtype region reading the parameters in place
        starts = torch.tensor([0] + sizes[:-1]).cumsum(0)
        row = torch.searchsorted(starts, gather, right=True) - 1
        code = torch.where(gather == fill, torch.full_like(gather, -1),
                           ((row.clamp_min(0) << 24) | (gather - starts[row.clamp_min(0)])))
        assert len(self.params) <= 63 and max(sizes) < (1 << 24)
        code = code.to(torch.int32).to(dev)
        self._maps = dict(dev=dev, gather=gather.to(dev), nbf=nbf, layout=layout, scaled=scaled,
                          code_bf=code[:nbf], code_f32=code[nbf:], tab=None, tab_key=None,
                          # fp32 engine: the conv weights gathered in fp32, then split (pack)
                          out_bf=torch.empty(nbf, dtype=torch.float32 if self.f32 else torch.bfloat16, device=dev),
                          out_f32=torch.empty(gather.numel() - nbf, dtype=torch.float32, device=dev),
                          glayout=glayout, gf1=gf1, gtotal=gtotal, ggather=torch.cat(gmaps).to(dev),
                          gscaled=gscaled, zero=torch.zeros(1, device=dev))

    def _src_table(self):
        M = self._maps
        key = tuple((p.data_ptr(), p.dtype, p.stride()) for p in self.params)
        if key != M["tab_key"]:
            rows = []
            for p in self.params:
                pad = 4 - p.dim()
                rows.append([p.data_ptr(), int(p.dtype == torch.bfloat16)] + [1] * pad + list(p.shape)
                            + [0] * pad + list(p.stride()))
            M["tab"] = torch.tensor(rows, dtype=torch.int64).to(M["dev"])
            M["tab_key"] = key
        return M["tab"]

    @torch.no_grad()
    def pack(self, dev):
        """Per-step weight packing (see _build_maps): two gather launches
        (csrc/wpack.hip: bf16 weights, fp32 biases / flow-encoder / flow-head
        weights) into persistent buffers, reading the parameters in place."""
        if self._maps is None or self._maps["dev"] != dev:
            self._build_maps(dev)
        M = self._maps
        nbf = M["nbf"]
        if all(p.dtype in (torch.float32, torch.bfloat16) and p.dim() <= 4 for p in self.params):
            tab = self._src_table()
            sc = M["scaled"]
            R.wpack_gather(M["code_bf"], tab, M["out_bf"], [a for a, _, _ in sc], [b for _, b, _ in sc],
                           [float(x) for _, _, x in sc])
            R.wpack_gather(M["code_f32"], tab, M["out_f32"], [], [], [])
            bf = M["out_bf"]
            vals = _Offset(M["out_f32"], nbf)
        else:  # reference path: cat + gather + cast
            src = torch.cat([p.detach().reshape(-1).float() for p in self.params] + [M["zero"]])
            v = src.index_select(0, M["gather"])
            for a, b, s in M["scaled"]:
                v[a:b].mul_(s)
            bf = v[:nbf] if self.f32 else v[:nbf].to(torch.bfloat16)
            vals = _Offset(v[nbf:], nbf)
        k = 1
        if self.f32:
            # every packed layout's last dim is a multiple of 32: one split of the
            # whole region into the F32 tiles' per-32-chunk [wh 32 | wl 32] rows
            v32 = bf.view(-1, 1, 32)
            hi = v32.to(torch.bfloat16)
            bf = torch.cat([hi, (v32 - hi.float()).to(torch.bfloat16)], 1).view(-1)
            k = 2
        ob, of = 0, nbf
        for pc, ws, wds, bs, hf, hdf in M["layout"]:
            n = ws.numel()
            pc.w = bf[k * ob:k * (ob + n)].view(ws[0], ws[1], k * ws[2])
            ob += n
            n = wds.numel()
            pc.wd = bf[k * ob:k * (ob + n)].view(wds[0], wds[1], k * wds[2])
            ob += n
            if self.f32 and _V3F_TRAIN:  # the fp32 weight-streaming tiles 81-83 read [frag(wh); frag(wl)]
                for t in (pc.w, pc.wd):
                    if frag32_eligible(t, pc.kh, pc.kw):
                        t._rs_frag32 = frag_weight_split(t)
            # fragment-major copies (bf16 engine): conv_fused finds them through
            # the packed weight's _rs_frag attribute when a weight-streaming tile (56-68) is chosen
            pc.wf = pc.wdf = None
            if hf:
                pc.wf = bf[ob:ob + ws.numel()].view(ws)
                ob += ws.numel()
                pc.w._rs_frag = pc.wf
            if hdf:
                pc.wdf = bf[ob:ob + wds.numel()].view(wds)
                ob += wds.numel()
                pc.wd._rs_frag = pc.wdf
            pc.b = vals[of:of + bs.numel()]
            of += bs.numel()
        fc = self.f1c
        self.f1w = vals[of:of + 49 * 2 * fc].view(7, 7, 2, fc)
        of += 49 * 2 * fc
        self.f1b = vals[of:of + fc]
        of += fc
        # 2-channel output conv (csrc/flowhead.hip): fp32 [2][3][3][Cin]
        fcw = self.model.update_block.flow_head.conv2.weight
        self.flow_w32 = vals[of:of + fcw.numel()].view(fcw.shape[0], fcw.shape[2], fcw.shape[3], fcw.shape[1])

    def side_stream(self, dev, slot: int = 0, flow: bool = False):
        from .raft import OVERLAP
        if not self.model.cfg.overlap_encoders or (flow and not OVERLAP["flow"]):
            return None
        return self.model._side_stream(dev, slot)

    def grad_buffers(self, dev):
        """One zero-filled fp32 buffer holding every packed gradient accumulator."""
        M = self._maps
        g = torch.zeros(M["gtotal"], device=dev)
        for pc, (dwo, dws, dbo, nb) in zip(self.convs, M["glayout"]):
            pc.dw = g[dwo:dwo + dws[0] * dws[1] * dws[2]].view(dws)
            pc.db = g[dbo:dbo + nb]
        a, b = M["gf1"]
        return g, g[a:b].view(49, 2, self.f1c), g[b:b + self.f1c]

    def unpack_grads(self, g):
        M = self._maps
        flat = g.index_select(0, M["ggather"])
        for a, b, s in M["gscaled"]:
            flat[a:b].mul_(s)
        out, o = [], 0
        for p in self.params:
            out.append(flat[o:o + p.numel()].view(p.shape))
            o += p.numel()
        return out

    @staticmethod
    def config_capable(cfg) -> bool:
        """The configuration half of ``eligible`` (no tensors needed): bf16
        (mixed precision) and fp32 training both run the fused engine."""
        return bool(cfg.fused_gru) and getattr(cfg, "fused_train", True)

    @staticmethod
    def eligible(model, image, corr_fn) -> bool:
        corr_ok = getattr(corr_fn, "state", None) is not None or (  # all-pairs pyramid, or on-the-fly (bf16)
            getattr(corr_fn, "f2s", None) is not None and corr_fn.radius == (3 if model.cfg.small else 4)
            and len(corr_fn.f2s) == 4 and corr_fn.f1.dtype == torch.bfloat16 and model.cfg.mixed_precision)
        return (image.device.type == "cuda" and torch.is_grad_enabled() and model.training
                and FusedTrainEngine.config_capable(model.cfg)
                and getattr(corr_fn, "hip", False) and corr_ok
                and _ext.use_hip(image))

    @staticmethod
    def corr_inputs(corr_fn):
        """(corr_state, token, otf tensors) for FusedTrainLoop.apply: the all-pairs
        pyramid state + its volume token, or the on-the-fly correlation's f1 and
        pooled f2 levels (their gradients are returned by the loop itself)."""
        if getattr(corr_fn, "state", None) is not None:
            return corr_fn.state, corr_fn.token, ()
        return None, None, (corr_fn.f1, *corr_fn.f2s)

    def buffers(self, B, H, W, iters, dev):
        key = (B, H, W, iters, dev)
        S = self._bufs.get(key)
        adt = self.adt
        if S is None and self.small:
            n = iters * B
            e = lambda b, c: torch.empty(b, H, W, c, device=dev, dtype=adt)
            z = lambda b, c: torch.zeros(b, H, W, c, device=dev, dtype=adt)
            S = dict(
                corr=e(n, SCORR_PAD), f1=e(n, 64), mot=e(n, 128),
                hx=z(n + B, 256),                 # channels 242:256 stay zero
                z=[e(n, SHD)], r=[e(n, SHD)], q=[e(n, SHD)],
                rh=[z(n, 128)],                   # channels 96:128 stay zero (weight-gradient window)
                head=e(n, 128), inp=e(B, 64),
                C=torch.empty(n + B, 2, H, W, device=dev),
                d_flow=torch.zeros(n, H, W, 64, device=dev, dtype=adt),  # 2 real
                # (padded K: d_q's channels 96:128 stay zero, relu_take zero-fills d_conv's 80:)
                d_head=e(n, 128), d_zr=[e(n, 2 * SHD)], d_q=[z(n, 128) if self.spad else e(n, SHD)],
                d_conv=e(n, 128 if self.spad else 96), d_mot=e(n, 128),
                d_f1=e(n, 64), d_corr=e(n, SCORR_PAD),
                G=torch.empty(B, H, W, 256, device=dev),
            )
            self._bufs = {key: S}
        elif S is None:
            n = iters * B
            e = lambda b, c: torch.empty(b, H, W, c, device=dev, dtype=adt)
            S = dict(
                corr=e(n, CORR_PAD), c1=e(n, 256), f1=e(n, 128), mot=e(n, 256), hx=e(n + B, 256), h1=e(n, HD),
                z=[e(n, HD), e(n, HD)], r=[e(n, HD), e(n, HD)], q=[e(n, HD), e(n, HD)], rh=[e(n, HD), e(n, HD)],
                head=e(n, 512), mask=e(n, 576), inp=e(B, 128),
                C=torch.empty(n + B, 2, H, W, device=dev),  # coords before iteration i = slot i
                # gradient (dY) slots (zero-initialised: only the leading channels are written)
                d_mask=torch.zeros(n, H, W, 640, device=dev, dtype=adt),
                d_flow=torch.zeros(n, H, W, 64, device=dev, dtype=adt),  # 2 real
                d_head=e(n, 512), d_zr=[e(n, 256), e(n, 256)], d_q=[e(n, HD), e(n, HD)], d_conv=e(n, 128),
                d_c2f2=e(n, 256), d_c1=e(n, 256), d_f1=e(n, 128), d_corr=e(n, CORR_PAD),
                G=torch.empty(B, H, W, 384, device=dev),
            )
            self._bufs = {key: S}  # one shape at a time (training crops are fixed)
        return S


def _split_bf16(t: torch.Tensor):
    """fp32 -> (hi, lo) bf16 with hi = bf16(t), lo = bf16(t - hi): one pass of
    csrc/split.hip for contiguous device tensors."""
    if t.is_cuda and t.is_contiguous() and t.data_ptr() % 16 == 0:
        hi, lo = R.split_bf16(t)
        return hi, lo
    hi = t.to(torch.bfloat16)
    return hi, (t - hi.float()).to(torch.bfloat16)


# csrc/wgrad_v3.hip (all taps per block, split-K partials reduced in order) for
# the 3x3 / 1x5 / 5x1 convs with more than 64 outputs; measured at the
# training shape (scripts/bench_conv.py --wgrad 12 --v3wgrad,
# profiles/r5/README.md): GRU z|r 400 -> 302 us, q 217 -> 171, head 475 -> 348,
# convc2 449 -> 387; the 64-output convf2 stays on conv_wgrad.hip (107 us).
_WG3 = True


def _wgrad_fn(pc, segs, bn128):
    if (_WG3 and pc.kh * pc.kw in (5, 9) and pc.cout > 64 and all(int(s[2]) % 64 == 0 for s in segs)):
        bm = 128 if pc.cout >= 512 else 64
        return lambda *a: R.wgrad_v3(*a, bm)
    return lambda *a: R.conv_wgrad(*a, bn128)


def _conv_wgrad(eng, pc, dy, yoff, segs, H, W, bn128=0):
    """``pc.dw += dY^T X`` (+ ``pc.db += colsum dY``) over every iteration's
    pixels on csrc/conv_wgrad.hip.  fp32 engine: the bf16 GEMM on the split
    operands, dYh.Xh + dYl.Xh + dYh.Xl (the bias sums of the first two give
    colsum(dYh + dYl))."""
    per = [s[0].shape[0] * H * W for s in segs]
    wg = _wgrad_fn(pc, segs, bn128)
    if not eng.f32:
        wg(dy, yoff, pc.cout, [s[0] for s in segs], [s[1] for s in segs], [s[2] for s in segs],
           per, pc.kh, pc.kw, pc.dw, pc.db)
        return
    cache = eng.__dict__.setdefault("_split_cache", {})
    def split(t):
        key = (t.data_ptr(), tuple(t.shape))
        v = cache.get(key)
        if v is None:
            v = cache[key] = _split_bf16(t)
        return v
    dyh, dyl = split(dy)
    xs = [split(s[0]) for s in segs]
    offs, chans = [s[1] for s in segs], [s[2] for s in segs]
    wg(dyh, yoff, pc.cout, [x[0] for x in xs], offs, chans, per, pc.kh, pc.kw, pc.dw, pc.db)
    wg(dyl, yoff, pc.cout, [x[0] for x in xs], offs, chans, per, pc.kh, pc.kw, pc.dw, pc.db)
    wg(dyh, yoff, pc.cout, [x[1] for x in xs], offs, chans, per, pc.kh, pc.kw, pc.dw, None)


class DeferGrads(torch.autograd.Function):
    """Identity on the update-block parameters, applied at the START of the
    RAFT forward (before the encoders).  Its backward therefore has the
    lowest autograd priority of the step and runs after the encoder backward
    passes: FusedTrainLoop.backward launches the iteration-batched weight
    gradients on the second HIP stream and returns at once, the encoders'
    backward runs on the main stream concurrently, and this node joins the
    streams before the gradients reach AccumulateGrad / DDP hooks / the
    optimizer."""

    @staticmethod
    def forward(ctx, stream, *params):
        ctx.stream = stream
        return tuple(p.view_as(p) for p in params)

    @staticmethod
    def backward(ctx, *grads):
        dev = next(g.device for g in grads if g is not None)
        torch.cuda.current_stream(dev).wait_stream(ctx.stream)
        return (None, *grads)


class _Offset:
    """fp32 values addressed in the packed gather's coordinates (the bf16
    region [0, nbf) precedes them): vals[a:b] -> t[a - nbf : b - nbf]."""
    __slots__ = ("t", "o")

    def __init__(self, t, o):
        self.t, self.o = t, o

    def __getitem__(self, s):
        return self.t[s.start - self.o:s.stop - self.o]


class FusedTrainLoop(torch.autograd.Function):
    """``otf``: None (all-pairs pyramid in corr_state) or (radius, scale, n_levels):
    the first n_levels + 1 of ``tensors`` are the on-the-fly correlation's f1 and
    pooled f2 levels (reference AlternateCorrBlock, core/corr.py:63-91, here also
    differentiable: SURVEY B1); the rest are the update-block parameters."""

    @staticmethod
    def forward(ctx, eng, corr_state, token, net, inp, coords0, coords1, iters, defer, otf, *tensors):
        nt = 0 if otf is None else otf[2] + 1
        otf_t, params = tensors[:nt], tensors[nt:]
        if eng.small:
            return _small_forward(ctx, eng, corr_state, net, inp, coords0, coords1, iters, defer, otf, otf_t)
        B, _, H, W = coords1.shape
        dev = coords1.device
        eng.pack(dev)
        f1w, f1b = eng.f1w, eng.f1b
        S = eng.buffers(B, H, W, iters, dev)
        sl = lambda t, i: t[i * B:(i + 1) * B]
        if inp is None:
            # net: the context encoder's raw output -- split + tanh / relu
            # (reference core/raft.py:108-110) straight into the slots, one pass
            cn = net.permute(0, 2, 3, 1).to(S["inp"].dtype).contiguous()
            R.context_act(cn, S["hx"][:B], S["inp"], HD)
        else:
            S["hx"][:B, ..., :HD].copy_(net.permute(0, 2, 3, 1))
            S["inp"].copy_(inp.permute(0, 2, 3, 1))
        C = S["C"]
        sl(C, 0).copy_(coords1.detach())
        c0 = coords0.detach().float().contiguous()
        inpb = S["inp"]
        if otf is not None:
            S["corr"][..., otf[2] * 81:].zero_()  # K padding of the correlation slot (lookup_into zeroes its own)
        # flow branch (flow encoder + convf2) on the second HIP stream, parallel
        # to lookup + convc1 + convc2; disjoint channels of `mot`, joined before
        # the conv that reads it
        main, side = torch.cuda.current_stream(dev), eng.side_stream(dev, flow=True)
        for i in range(iters):
            hx, hx1 = sl(S["hx"], i), sl(S["hx"], i + 1)
            coords = sl(C, i)
            if side is not None:
                side.wait_stream(main)
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                R.flow_encode(coords, f1w, f1b, sl(S["f1"], i), 0, hx, 254)
                conv_fused([(sl(S["f1"], i), 0, 128)], eng.f2.w, eng.f2.b, 3, 3, 64, EPI_RELU, sl(S["mot"], i), 192)
            if otf is None:
                R.corr_lookup_into(corr_state.pyr, coords, corr_state.radius, sl(S["corr"], i))
            else:
                cf = R.corr_otf(otf_t[0], list(otf_t[1:]), coords, otf[0], otf[1], True)
                sl(S["corr"], i)[..., :cf.shape[-1]].copy_(cf)
            conv_fused([(sl(S["corr"], i), 0, CORR_PAD)], eng.c1.w, eng.c1.b, 1, 1, 256, EPI_RELU, sl(S["c1"], i))
            conv_fused([(sl(S["c1"], i), 0, 256)], eng.c2.w, eng.c2.b, 3, 3, 192, EPI_RELU, sl(S["mot"], i), 0)
            if side is not None:
                main.wait_stream(side)
            conv_fused([(sl(S["mot"], i), 0, 256)], eng.cv.w, eng.cv.b, 3, 3, 126, EPI_RELU, hx, HD)
            h_in = [(hx, 0), (sl(S["h1"], i), 0)]
            h_out = [(sl(S["h1"], i), 0), (hx1, 0)]
            for p in range(2):
                hb, ho = h_in[p]
                z, r, q, rh = (sl(S[k][p], i) for k in ("z", "r", "q", "rh"))
                conv_fused([(hb, ho, HD), (inpb, 0, 128), (hx, HD, 128)], eng.zr[p].w, eng.zr[p].b, eng.zr[p].kh,
                           eng.zr[p].kw, 2 * HD, EPI_GRU_ZR, z, 0, hd=HD, out2=rh, out3=r, aux1=hb, a1off=ho)
                ob, oo = h_out[p]
                conv_fused([(rh, 0, HD), (inpb, 0, 128), (hx, HD, 128)], eng.q[p].w, eng.q[p].b, eng.q[p].kh,
                           eng.q[p].kw, HD, EPI_GRU_Q, ob, oo, out2=q, aux1=hb, a1off=ho, aux2=z)
            head = sl(S["head"], i)
            conv_fused([(hx1, 0, HD)], eng.head.w, eng.head.b, 3, 3, 512, EPI_RELU, head, 0)
            # coords_{i+1} = coords_i + delta (out of place: the history is kept for backward)
            R.flow_head(head, 0, 256, eng.flow_w32, eng.flow.b, sl(C, i + 1), coords)
            conv_fused([(head, 256, 256)], eng.mask2.w, eng.mask2.b, 1, 1, 576, EPI_SCALE, sl(S["mask"], i), 0,
                       scale=0.25)
        # every iteration's convex upsampling in one launch (they do not feed back)
        n = iters * B
        flows = (C[B:].view(iters, B, 2, H, W) - c0).view(n, 2, H, W)
        up = R.convex_upsample(flows, S["mask"])
        ctx.eng, ctx.state, ctx.S, ctx.iters = eng, corr_state, S, iters
        ctx.otf = otf
        if otf is not None:
            ctx.save_for_backward(*otf_t)
        ctx.defer = bool(defer) and eng.side_stream(dev) is not None
        ctx.c0 = c0
        ctx.net_dtype = net.dtype
        ctx.inp_dtype = inp.dtype if inp is not None else None  # None: net was the raw context output
        return up

    @staticmethod
    def backward(ctx, g_up):
        if ctx.eng.small:
            return _small_backward(ctx, g_up)
        eng, st, S, iters = ctx.eng, ctx.state, ctx.S, ctx.iters
        c0 = ctx.c0
        B, H, W = S["inp"].shape[:3]
        dev = c0.device
        n = iters * B
        sl = lambda t, i: t[i * B:(i + 1) * B]
        main = torch.cuda.current_stream(dev)
        # deferred: convf2 dgrad + all weight gradients on their own stream
        # (joined by DeferGrads.backward); else convf2 dgrad on the side stream
        side = eng.side_stream(dev, 1 if ctx.defer else 0, flow=not ctx.defer)
        lside = eng.side_stream(dev, 0) if ctx.defer else None
        otf = ctx.otf
        if otf is None:
            if st.gpyr is None:
                st.gpyr = st.zero_grads()
        else:
            otf_t = ctx.saved_tensors
            d_otf = None  # fp32 sums over the iterations: [df1, df2_0 .. df2_{L-1}]
        G = S["G"]
        G.zero_()
        inpb = S["inp"]
        C = S["C"]
        if g_up is None:
            g_up = torch.zeros(n, 2, 8 * H, 8 * W, device=dev)
        flows = (C[B:].view(iters, B, 2, H, W) - c0).view(n, 2, H, W)
        # the mask gradient straight into the padded d_mask slots (channels 576.. stay zero)
        dflow, _ = R.convex_upsample_backward(flows, S["mask"], g_up.contiguous(), S["d_mask"])
        S["d_flow"][..., :2].copy_(dflow.permute(0, 2, 3, 1))
        for i in reversed(range(iters)):
            hx, hx1, head = sl(S["hx"], i), sl(S["hx"], i + 1), sl(S["head"], i)
            dm, df, dh = sl(S["d_mask"], i), sl(S["d_flow"], i), sl(S["d_head"], i)
            conv_fused([(dm, 0, 576)], eng.mask2.wd, None, 1, 1, 256, EPI_RELU_BWD, dh, 256, aux1=head, a1off=256)
            R.flow_head_dgrad(sl(dflow, i), eng.flow_w32, 256, head, 0, dh, 0)
            conv_fused([(dh, 0, 512)], eng.head.wd, None, 3, 3, HD, EPI_ACC_F32, G, 0)
            h_in = [(hx, 0), (sl(S["h1"], i), 0)]
            for p in (1, 0):
                hb, ho = h_in[p]
                z, r, q = sl(S["z"][p], i), sl(S["r"][p], i), sl(S["q"][p], i)
                dq, dzr = sl(S["d_q"][p], i), sl(S["d_zr"][p], i)
                R.gru_gate_bwd(G, z, q, hb, ho, dq, dzr)
                conv_fused([(dq, 0, HD)], eng.q[p].wd, None, eng.q[p].kh, eng.q[p].kw, 384, EPI_GRU_QBWD, G, 0,
                           hd=HD, out2=dzr, o2off=HD, aux1=hb, a1off=ho, aux2=r)
                conv_fused([(dzr, 0, 256)], eng.zr[p].wd, None, eng.zr[p].kh, eng.zr[p].kw, 384, EPI_ACC_F32, G, 0)
            dcv = sl(S["d_conv"], i)
            R.relu_take(G, 256, 126, 128, hx, HD, dcv)
            dc2f2 = sl(S["d_c2f2"], i)
            conv_fused([(dcv, 0, 128)], eng.cv.wd, None, 3, 3, 256, EPI_RELU_BWD, dc2f2, 0, aux1=sl(S["mot"], i))
            dc1 = sl(S["d_c1"], i)
            if side is not None:  # convf2 dgrad (only feeds the flow-encoder wgrad) on the side stream
                side.wait_stream(main)
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                conv_fused([(dc2f2, 192, 64)], eng.f2.wd, None, 3, 3, 128, EPI_RELU_BWD, sl(S["d_f1"], i), 0,
                           aux1=sl(S["f1"], i))
            conv_fused([(dc2f2, 0, 192)], eng.c2.wd, None, 3, 3, 256, EPI_RELU_BWD, dc1, 0, aux1=sl(S["c1"], i))
            dcorr = sl(S["d_corr"], i)
            conv_fused([(dc1, 0, 256)], eng.c1.wd, None, 1, 1, CORR_PAD, EPI_BIAS, dcorr, 0)
            # the pyramid-gradient scatter only feeds the correlation backward after the
            # loop: on its own stream (per-iteration d_corr slots, in-order accumulation)
            if lside is not None:
                lside.wait_stream(main)
            with torch.cuda.stream(lside) if lside is not None else contextlib.nullcontext():
                if otf is None:
                    R.corr_lookup_backward(st.gpyr, sl(C, i), st.radius, dcorr)
                else:
                    ch = otf[2] * 81
                    gi = R.corr_otf_backward(otf_t[0], list(otf_t[1:]), sl(C, i), otf[0], otf[1],
                                             dcorr[..., :ch].contiguous())
                    if d_otf is None:
                        d_otf = list(gi)
                    else:
                        for acc, g in zip(d_otf, gi):
                            acc.add_(g)
        if lside is not None:
            main.wait_stream(lside)
            if otf is not None:
                for g in d_otf:
                    g.record_stream(main)
        if otf is None and _EARLY_CORR_BWD:
            st.early_backward()
        if ctx.inp_dtype is None:  # adjoint of context_act: the raw context output's gradient, one pass
            d_net = R.context_act_backward(G, S["hx"][:B], S["inp"], HD).permute(0, 3, 1, 2).to(ctx.net_dtype)
            d_inp = None
        else:
            d_net = G[..., :HD].permute(0, 3, 1, 2).to(ctx.net_dtype)
            d_inp = G[..., HD:HD + 128].permute(0, 3, 1, 2).to(ctx.inp_dtype)

        grads = FusedTrainLoop._param_grads(ctx, FusedTrainLoop._wgrads, S, C, B, H, W, n, main, side)
        if otf is None:
            token_grad, otf_grads = torch.zeros((), device=dev), ()
        else:
            token_grad = None
            otf_grads = tuple(g.to(t.dtype) for g, t in zip(d_otf, otf_t))
        return (None, None, token_grad, d_net, d_inp, None, None, None, None, None, *otf_grads, *grads)

    @staticmethod
    def _param_grads(ctx, wgrads, S, C, B, H, W, n, main, side):
        """Weight / bias gradients batched over all iterations (``wgrads``), the
        data-parallel all-reduce of the packed buffer and the unpacking --
        deferred onto the weight-gradient stream when ``ctx.defer``."""
        eng = ctx.eng
        gbuf, dwf, dbf = eng.grad_buffers(main.device)
        if ctx.defer:  # on the weight-gradient stream, joined by DeferGrads.backward
            side.wait_stream(main)
            gbuf.record_stream(side)
            wstream = torch.cuda.stream(side)
        else:
            if side is not None:
                main.wait_stream(side)
            wstream = contextlib.nullcontext()
        with wstream:
            wgrads(eng, S, C, gbuf, dwf, dbf, B, H, W, n)
            eng.__dict__.pop("_split_cache", None)  # fp32 engine: the split operands of this step
            if eng.grad_group is not None:  # data parallel: one RCCL all-reduce of the packed buffer
                eng.reduce_packed(gbuf)
            grads = [gr if gr.dtype == p.dtype else gr.to(p.dtype)
                     for gr, p in zip(eng.unpack_grads(gbuf), eng.params)]
        if ctx.defer:
            for gr in grads:
                gr.record_stream(main)
        return grads

    @staticmethod
    def _wgrads(eng, S, C, gbuf, dwf, dbf, B, H, W, n):
        inpb = S["inp"]
        hxs = S["hx"][:n]

        def wg(pc, dy, yoff, segs, bn128=0):
            # weight gradient + fused bias gradient (column sums of dY); tile
            # variant per conv where it measured faster (scripts/bench_conv.py
            # --wgrad 12 at the training shape: 8-wave 256x64 for the 3x3
            # 256->192 conv 475 -> 397 us and GRU z|r 404 -> 374 us, 8-wave
            # 128x128 for the 128->512 head 472 -> 425 us)
            _conv_wgrad(eng, pc, dy, yoff, segs, H, W, bn128)

        wg(eng.mask2, S["d_mask"], 0, [(S["head"], 256, 256)])
        wg(eng.flow, S["d_flow"], 0, [(S["head"], 0, 256)])
        wg(eng.head, S["d_head"], 0, [(S["hx"][B:], 0, HD)], 2)
        hins = [hxs, S["h1"]]
        for p in range(2):
            wg(eng.zr[p], S["d_zr"][p], 0, [(hins[p], 0, HD), (inpb, 0, 128), (hxs, HD, 128)], 4)
            wg(eng.q[p], S["d_q"][p], 0, [(S["rh"][p], 0, HD), (inpb, 0, 128), (hxs, HD, 128)])
        wg(eng.cv, S["d_conv"], 0, [(S["mot"], 0, 256)], 2)  # 8-wave 128x128: 238 vs 258 us (profiles/r4/wgrad_bench_s21.log)
        wg(eng.c2, S["d_c2f2"], 0, [(S["c1"], 0, 256)], 4)
        wg(eng.f2, S["d_c2f2"], 192, [(S["f1"], 0, 128)])
        wg(eng.c1, S["d_c1"], 0, [(S["corr"], 0, CORR_PAD)])
        R.flow_wgrad(C[:n], S["d_f1"], dwf, dbf)


# ------------------------------------------------------------------ RAFT-small
# The same engine for the small model (reference core/update.py:
# SmallMotionEncoder, ConvGRU 3x3 hidden 96, FlowHead(96, 128), no mask:
# bilinear x8 upsampling, core/raft.py:134-137).  Per iteration:
#   flow branch (side stream): flow_encode -> f1 (64), convf2 3x3 -> mot[96:128]
#   lookup (radius 3, 196 taps) -> corr, convc1 1x1 -> mot[0:96]
#   conv 3x3 mot -> hx[160:240]           hx = [h | inp | motion | flow | 0]
#   z|r 3x3 over hx[0:256] (gate epilogue), q 3x3 over [r*h | hx[96:256]] -> h'
#   head 3x3 h' -> 128 (ReLU), flow head -> coords_{i+1}
# All iterations' x8 upsamplings are one interpolation after the loop.

_INTERP = {}


def _interp_matrix(n_in: int, n_out: int, dev) -> torch.Tensor:
    """[n_out, n_in] weights of 1-D linear interpolation with align_corners=True,
    using upsample_bilinear2d's float32 source-index arithmetic."""
    key = (n_in, n_out, str(dev))
    m = _INTERP.get(key)
    if m is None:
        scale = torch.tensor(float(n_in - 1), dtype=torch.float32) / (n_out - 1) if n_out > 1 else torch.tensor(0.0)
        src = scale * torch.arange(n_out, dtype=torch.float32)
        i0 = src.long()
        lam = src - i0.float()
        i1 = torch.where(i0 < n_in - 1, i0 + 1, i0)
        m = torch.zeros(n_out, n_in, dtype=torch.float32)
        rows = torch.arange(n_out)
        m[rows, i0] += 1 - lam
        m[rows, i1] += lam
        m = _INTERP[key] = m.to(dev)
    return m


def _small_forward(ctx, eng, corr_state, net, inp, coords0, coords1, iters, defer, otf=None, otf_t=()):
    """``otf``: None (all-pairs pyramid) or (radius 3, scale, 4 levels) with
    ``otf_t`` = (f1, pooled f2 levels): the on-the-fly correlation (reference
    AlternateCorrBlock with RAFT-small's radius, core/raft.py:29-33)."""
    B, _, H, W = coords1.shape
    dev = coords1.device
    hd = SHD
    eng.pack(dev)
    S = eng.buffers(B, H, W, iters, dev)
    sl = lambda t, i: t[i * B:(i + 1) * B]
    hv = S["hx"].view(iters + 1, B, H, W, 256)
    hv[0, ..., :hd].copy_(net.permute(0, 2, 3, 1))
    hv[..., hd:hd + 64].copy_(inp.permute(0, 2, 3, 1))  # the context features of every slot
    C = S["C"]
    sl(C, 0).copy_(coords1.detach())
    c0 = coords0.detach().float().contiguous()
    if otf is not None:
        S["corr"][..., otf[2] * 49:].zero_()  # K padding of the correlation slot (lookup_into zeroes its own)
    main, side = torch.cuda.current_stream(dev), eng.side_stream(dev, flow=True)
    zr, q = eng.zr[0], eng.q[0]
    for i in range(iters):
        hx, hx1 = sl(S["hx"], i), sl(S["hx"], i + 1)
        coords = sl(C, i)
        mot = sl(S["mot"], i)
        if side is not None:
            side.wait_stream(main)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            R.flow_encode(coords, eng.f1w, eng.f1b, sl(S["f1"], i), 0, hx, 240)
            conv_fused([(sl(S["f1"], i), 0, 64)], eng.f2.w, eng.f2.b, 3, 3, 32, EPI_RELU, mot, 96)
        if otf is None:
            R.corr_lookup_into(corr_state.pyr, coords, corr_state.radius, sl(S["corr"], i))
        else:
            cf = R.corr_otf(otf_t[0], list(otf_t[1:]), coords, otf[0], otf[1], True)
            sl(S["corr"], i)[..., :cf.shape[-1]].copy_(cf)
        conv_fused([(sl(S["corr"], i), 0, SCORR_PAD)], eng.c1.w, eng.c1.b, 1, 1, hd, EPI_RELU, mot, 0)
        if side is not None:
            main.wait_stream(side)
        conv_fused([(mot, 0, 128)], eng.cv.w, eng.cv.b, 3, 3, 80, EPI_RELU, hx, 160)
        z, r, qq, rh = (sl(S[k][0], i) for k in ("z", "r", "q", "rh"))
        conv_fused([(hx, 0, 256)], zr.w, zr.b, 3, 3, 2 * hd, EPI_GRU_ZR, z, 0, hd=hd, out2=rh, out3=r,
                   aux1=hx, a1off=0)
        qseg = [(rh, 0, 128), (hx, 64, 192)] if eng.spad else [(rh, 0, hd), (hx, hd, 160)]
        conv_fused(qseg, q.w, q.b, 3, 3, hd, EPI_GRU_Q, hx1, 0, out2=qq, aux1=hx, a1off=0, aux2=z)
        head = sl(S["head"], i)
        conv_fused([(hx1, 0, 128 if eng.spad else hd)], eng.head.w, eng.head.b, 3, 3, 128, EPI_RELU, head, 0)
        R.flow_head(head, 0, 128, eng.flow_w32, eng.flow.b, sl(C, i + 1), coords)
    n = iters * B
    flows = (C[B:].view(iters, B, 2, H, W) - c0).view(n, 2, H, W)
    up = 8 * torch.nn.functional.interpolate(flows, size=(8 * H, 8 * W), mode="bilinear", align_corners=True)
    ctx.eng, ctx.state, ctx.S, ctx.iters, ctx.otf = eng, corr_state, S, iters, otf
    if otf is not None:
        ctx.save_for_backward(*otf_t)
    ctx.defer = bool(defer) and eng.side_stream(dev) is not None
    ctx.c0 = c0
    ctx.net_dtype, ctx.inp_dtype = net.dtype, inp.dtype
    return up


def _small_backward(ctx, g_up):
    eng, st, S, iters = ctx.eng, ctx.state, ctx.S, ctx.iters
    hd = SHD
    B, H, W = S["inp"].shape[:3]
    dev = ctx.c0.device
    n = iters * B
    sl = lambda t, i: t[i * B:(i + 1) * B]
    main = torch.cuda.current_stream(dev)
    side = eng.side_stream(dev, 1 if ctx.defer else 0, flow=not ctx.defer)
    lside = eng.side_stream(dev, 0) if ctx.defer else None
    otf = ctx.otf
    if otf is None:
        if st.gpyr is None:
            st.gpyr = st.zero_grads()
    else:
        otf_t = ctx.saved_tensors
        d_otf = None  # fp32 sums over the iterations: [df1, df2_0 .. df2_3]
    G = S["G"]  # fp32 [dh 96 | d inp 64 | d motion 80 | d flow 2 | 0]
    G.zero_()
    C = S["C"]
    if g_up is None:
        g_up = torch.zeros(n, 2, 8 * H, 8 * W, device=dev)
    # adjoint of the x8 bilinear upsampling (align_corners) of every iteration:
    # a gather kernel over the interpolation matrices' bands (csrc/convex_upsample.hip
    # upflow8_bwd_kernel; deterministic, unlike the atomic scatter of
    # upsample_bilinear2d_backward)
    ah, aw = _interp_matrix(H, 8 * H, dev), _interp_matrix(W, 8 * W, dev)
    dflow = torch.ops.raft_stir.upflow8_backward(g_up.float().contiguous(), ah, aw)
    S["d_flow"][..., :2].copy_(dflow.permute(0, 2, 3, 1))
    zr, q = eng.zr[0], eng.q[0]
    for i in reversed(range(iters)):
        hx, head, dh = sl(S["hx"], i), sl(S["head"], i), sl(S["d_head"], i)
        R.flow_head_dgrad(sl(dflow, i), eng.flow_w32, 128, head, 0, dh, 0)
        conv_fused([(dh, 0, 128)], eng.head.wd, None, 3, 3, hd, EPI_ACC_F32, G, 0)
        z, r, qq = sl(S["z"][0], i), sl(S["r"][0], i), sl(S["q"][0], i)
        dq, dzr = sl(S["d_q"][0], i), sl(S["d_zr"][0], i)
        R.gru_gate_bwd(G, z, qq, hx, 0, dq, dzr)
        conv_fused([(dq, 0, q.cy)], q.wd, None, 3, 3, 256, EPI_GRU_QBWD, G, 0, hd=hd, out2=dzr, o2off=hd,
                   aux1=hx, a1off=0, aux2=r)
        conv_fused([(dzr, 0, 2 * hd)], zr.wd, None, 3, 3, 256, EPI_ACC_F32, G, 0)
        dcv, dmot = sl(S["d_conv"], i), sl(S["d_mot"], i)
        R.relu_take(G, 160, 80, 96, hx, 160, dcv)  # consumes d motion, drops d flow (coords detached)
        conv_fused([(dcv, 0, eng.cv.cy)], eng.cv.wd, None, 3, 3, 128, EPI_RELU_BWD, dmot, 0, aux1=sl(S["mot"], i))
        if side is not None:
            side.wait_stream(main)
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            conv_fused([(dmot, 96, 32)], eng.f2.wd, None, 3, 3, 64, EPI_RELU_BWD, sl(S["d_f1"], i), 0,
                       aux1=sl(S["f1"], i))
        dcorr = sl(S["d_corr"], i)
        conv_fused([(dmot, 0, eng.c1.cy)], eng.c1.wd, None, 1, 1, SCORR_PAD, EPI_BIAS, dcorr, 0)
        if lside is not None:
            lside.wait_stream(main)
        with torch.cuda.stream(lside) if lside is not None else contextlib.nullcontext():
            if otf is None:
                R.corr_lookup_backward(st.gpyr, sl(C, i), st.radius, dcorr)
            else:
                gi = R.corr_otf_backward(otf_t[0], list(otf_t[1:]), sl(C, i), otf[0], otf[1],
                                         dcorr[..., :otf[2] * 49].contiguous())
                if d_otf is None:
                    d_otf = list(gi)
                else:
                    for acc, g in zip(d_otf, gi):
                        acc.add_(g)
    if lside is not None:
        main.wait_stream(lside)
        if otf is not None:
            for g in d_otf:
                g.record_stream(main)
    if otf is None and _EARLY_CORR_BWD:
        st.early_backward()
    d_net = G[..., :hd].permute(0, 3, 1, 2).to(ctx.net_dtype)
    d_inp = G[..., hd:hd + 64].permute(0, 3, 1, 2).to(ctx.inp_dtype)
    grads = FusedTrainLoop._param_grads(ctx, _small_wgrads, S, C, B, H, W, n, main, side)
    if otf is None:
        token_grad, otf_grads = torch.zeros((), device=dev), ()
    else:
        token_grad = None
        otf_grads = tuple(g.to(t.dtype) for g, t in zip(d_otf, otf_t))
    return (None, None, token_grad, d_net, d_inp, None, None, None, None, None, *otf_grads, *grads)


def _small_wgrads(eng, S, C, gbuf, dwf, dbf, B, H, W, n):
    hxs = S["hx"][:n]

    def wg(pc, dy, yoff, segs, bn128=0):
        _conv_wgrad(eng, pc, dy, yoff, segs, H, W, bn128)

    wg(eng.flow, S["d_flow"], 0, [(S["head"], 0, 128)])
    wg(eng.head, S["d_head"], 0, [(S["hx"][B:], 0, 128)])
    wg(eng.zr[0], S["d_zr"][0], 0, [(hxs, 0, 256)])
    wg(eng.q[0], S["d_q"][0], 0, [(S["rh"][0], 0, 128), (hxs, 64, 192)])
    wg(eng.cv, S["d_conv"], 0, [(S["mot"], 0, 128)])
    wg(eng.f2, S["d_mot"], 96, [(S["f1"], 0, 64)])
    wg(eng.c1, S["d_mot"], 0, [(S["corr"], 0, SCORR_PAD)])
    R.flow_wgrad(C[:n], S["d_f1"], dwf, dbf)
