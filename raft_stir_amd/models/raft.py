"""RAFT: Recurrent All-Pairs Field Transforms, MI355X engine.

Public API identical to reference core/raft.py:24-144:
    model = RAFT(args)             # args: Namespace with .small, .mixed_precision, ...
    flow_predictions = model(image1, image2, iters=12)                  # training
    flow_low, flow_up = model(image1, image2, iters=12, test_mode=True)  # inference
    model.freeze_bn()
and the same ``state_dict`` keys (fnet/cnet/update_block...), so reference
``.pth`` checkpoints (with or without the DataParallel ``module.`` prefix, see
raft_stir_amd.train.checkpoint) load unchanged.

Engine differences (outputs unchanged):
  * GPU: channels_last activations, bf16 autocast when ``mixed_precision``
    (the reference used fp16 AMP), all-pairs volume + pyramid from one MFMA
    kernel, HIP pyramid lookup, fused ConvGRU gates, HIP convex upsampler.
  * test_mode computes the mask head and the convex upsampling only on the
    last iteration -- the only one whose output is returned (reference B7).
  * GPU inference (no autograd, bf16) runs the refinement loop through the
    fused engine of models/fused_update.py: ~12 hand-written HIP launches per
    iteration over persistent NHWC buffers instead of the module graph.
  * GPU training (full RAFT and RAFT-small, bf16) runs it as ONE autograd node
    (models/fused_train.py): fused forward kernels saving activations, a
    hand-written backward (dgrad convs with gradient epilogues, gate
    backward kernels) and weight gradients batched over all iterations.
"""
from __future__ import annotations

import contextlib

import torch
import torch.nn as nn

from ..config import RAFTConfig, resolve_config
from ..ops import _ext
from ..ops import enc_conv
from ..ops import gru as gru_ops
from ..ops import wpack
from ..ops import reference as ref
from ..ops.upsample import convex_upsample, upflow8
from .corr import CorrBlock, AlternateCorrBlock
from .extractor import BasicEncoder, SmallEncoder
from .fused_encoder import FusedEncoders
from .fused_update import FusedUpdate
from .fused_train import DeferGrads, FusedTrainEngine, FusedTrainLoop
from .update import BasicUpdateBlock, SmallUpdateBlock


class _StreamHandoff(torch.autograd.Function):
    """Identity moving a tensor produced on `side` to the current stream.
    Marks the forward value as used by the current stream and the incoming
    gradient (allocated on the current stream) as used by `side`, where the
    producer's backward consumes it, so the caching allocator never hands
    either block to the other stream while a kernel still reads it."""

    @staticmethod
    def forward(ctx, x, side):
        ctx.side = side
        x.record_stream(torch.cuda.current_stream(x.device))
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g.record_stream(ctx.side)
        return g, None


_SIDE_STREAMS = {}  # (device index, slot) -> extra HIP stream
_FUSED_PREP = True  # one-kernel input normalisation into the fnet batch
_GRID_CACHE: dict = {}  # (h, w, device) -> (1, 2, h, w) pixel-coordinate grid (initialize_flow)
# per-mechanism switches of the multi-stream schedule (all gated by cfg.overlap_encoders)
# defer_enc (encoder conv weight gradients on the deferred stream too) is off:
# paired A/B on one box, 3 x 30 steps: 352 pairs/s on vs 366 off (the third
# stream then ends the backward late and its GEMMs contend with the dgrads)
# defer_enc re-measured in round 5: 405 vs 427 pairs/s (profiles/r5/ab_defer_enc_s32.txt)
OVERLAP = {"cnet": True, "flow": True, "defer": True, "defer_enc": False}


class _SplitPair(torch.autograd.Function):
    """``torch.split(x, [n, len(x) - n])`` whose backward returns the two
    gradients' common buffer when they are adjacent halves of one tensor with
    the same strides (the correlation backward writes d fmap1 / d fmap2 that
    way, csrc/ops.cpp corr_volume_backward) instead of concatenating them; a
    missing half's gradient is zeros of that half's shape (from ctx.shape)."""

    @staticmethod
    def forward(ctx, x, n):
        ctx.n, ctx.shape = n, x.shape
        return x[:n], x[n:]

    @staticmethod
    def backward(ctx, g1, g2):
        n, shape = ctx.n, ctx.shape
        if g1 is None and g2 is None:
            return None, None
        if g1 is None or g2 is None:
            z = g2 if g1 is None else g1
            if g1 is None:
                g1 = torch.zeros((n,) + tuple(shape[1:]), device=z.device, dtype=z.dtype)
            else:
                g2 = torch.zeros((shape[0] - n,) + tuple(shape[1:]), device=z.device, dtype=z.dtype)
        assert tuple(g1.shape) == (n,) + tuple(shape[1:]) and tuple(g2.shape) == (shape[0] - n,) + tuple(shape[1:])
        if (g1.dtype == g2.dtype and g1.stride() == g2.stride() and g1.untyped_storage().data_ptr()
                == g2.untyped_storage().data_ptr()
                and g2.storage_offset() == g1.storage_offset() + g1.shape[0] * g1.stride(0)):
            return g1.as_strided((g1.shape[0] + g2.shape[0],) + tuple(g1.shape[1:]), g1.stride(),
                                 g1.storage_offset()), None
        return torch.cat([g1, g2], 0), None


class RAFT(nn.Module):
    def __init__(self, args=None, **overrides):
        super().__init__()
        cfg = args if isinstance(args, RAFTConfig) else resolve_config(args, **overrides)
        self.cfg = cfg
        self.args = args if args is not None else cfg
        self.hidden_dim = hdim = cfg.hidden_dim
        self.context_dim = cdim = cfg.context_dim
        if cfg.small:
            self.fnet = SmallEncoder(output_dim=cfg.fnet_dim, norm_fn="instance", dropout=cfg.dropout)
            self.cnet = SmallEncoder(output_dim=hdim + cdim, norm_fn="none", dropout=cfg.dropout)
            self.update_block = SmallUpdateBlock(cfg, hidden_dim=hdim)
        else:
            self.fnet = BasicEncoder(output_dim=cfg.fnet_dim, norm_fn="instance", dropout=cfg.dropout)
            self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn="batch", dropout=cfg.dropout)
            self.update_block = BasicUpdateBlock(cfg, hidden_dim=hdim)
        self.set_fused_gru(cfg.fused_gru)
        if cfg.deterministic:  # process-wide switch (runtime/determinism.py)
            from ..runtime.determinism import set_deterministic
            set_deterministic(True)

    # ------------------------------------------------------------------ utils
    def set_fused_gru(self, enabled: bool):
        for m in self.modules():
            if hasattr(m, "fused") and m is not self:
                m.fused = enabled

    def _encoder_conv_params(self):
        """Weights (and biases) of the encoder convolutions, in a fixed order."""
        ps = self.__dict__.get("_enc_params")
        if ps is None or ps[0] is not self.fnet.conv1.weight:
            ps = []
            for enc in (self.fnet, self.cnet):
                for m in enc.modules():
                    if isinstance(m, nn.Conv2d):
                        ps.append(m.weight)
                        if m.bias is not None:
                            ps.append(m.bias)
            self.__dict__["_enc_params"] = ps
        return ps

    def _train_engine(self):
        eng = self.__dict__.get("_fused_train")
        if eng is None or eng.model is not self:
            eng = FusedTrainEngine(self)
            self.__dict__["_fused_train"] = eng
        return eng

    def _encoder_engine(self):
        eng = self.__dict__.get("_fused_enc")
        if eng is None or eng.model is not self:
            eng = FusedEncoders(self)
            self.__dict__["_fused_enc"] = eng
        return eng

    def _fused_engine(self):
        eng = self.__dict__.get("_fused")
        if eng is None or eng.model is not self:
            eng = FusedUpdate(self)
            self.__dict__["_fused"] = eng
        return eng

    @staticmethod
    def _side_stream(dev, slot: int = 0):
        """slot 0: context encoder / flow branch; slot 1: deferred weight gradients."""
        st = _SIDE_STREAMS.get((dev.index, slot))
        if st is None:
            st = _SIDE_STREAMS[(dev.index, slot)] = torch.cuda.Stream(device=dev)
        return st

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def initialize_flow(self, img):
        N, _, H, W = img.shape
        if img.device.type != "cuda" or torch.jit.is_tracing():
            c0 = ref.coords_grid(N, H // 8, W // 8, device=img.device)
            c1 = ref.coords_grid(N, H // 8, W // 8, device=img.device)
            return c0, c1
        # one cached (1, 2, h, w) grid per shape, expanded into two fresh
        # tensors: two copy kernels per forward instead of eight (arange x4,
        # stack, repeat); not cached while a hipGraph is being captured (its
        # memory would belong to the graph's pool)
        key = (H // 8, W // 8, img.device)
        g = _GRID_CACHE.get(key)
        if g is None:
            g = ref.coords_grid(1, H // 8, W // 8, device=img.device)
            if not torch.cuda.is_current_stream_capturing():
                _GRID_CACHE[key] = g
        shape = (N,) + tuple(g.shape[1:])
        return g.expand(shape).clone(), g.expand(shape).clone()

    def upsample_flow(self, flow, mask):
        return convex_upsample(flow, mask)

    def _autocast(self, device):
        enabled = bool(self.cfg.mixed_precision) and device.type == "cuda"
        return torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=enabled)

    # ---------------------------------------------------------------- forward
    def forward(self, image1, image2, iters=12, flow_init=None, upsample=True, test_mode=False):
        dev = image1.device
        gpu = dev.type == "cuda"
        xin = None
        if (gpu and _FUSED_PREP and image1.dtype == torch.float32 and image2.dtype == torch.float32
                and image1.shape == image2.shape and not (image1.requires_grad or image2.requires_grad)):
            # one kernel per image: x * 2/255 - 1 written straight into the two
            # halves of ONE channels-last buffer -- the feature encoder's batched
            # input (no separate scale / shift / layout-copy / cat kernels)
            B = image1.shape[0]
            xin = torch.empty((2 * B,) + tuple(image1.shape[1:]), device=dev,
                              memory_format=torch.channels_last)
            m1 = torch.tensor(-1.0)
            torch.add(m1, image1, alpha=2.0 / 255.0, out=xin[:B])
            torch.add(m1, image2, alpha=2.0 / 255.0, out=xin[B:])
            image1, image2 = xin[:B], xin[B:]
        else:
            image1 = 2 * (image1 / 255.0) - 1.0
            image2 = 2 * (image2 / 255.0) - 1.0
            fmt = torch.channels_last if gpu else torch.contiguous_format
            image1 = image1.contiguous(memory_format=fmt)
            image2 = image2.contiguous(memory_format=fmt)
        hdim, cdim = self.hidden_dim, self.context_dim
        mixed = bool(self.cfg.mixed_precision) and gpu

        # ONE autocast region for the whole forward: autocast caches the bf16
        # copy of every weight for the region, so each conv weight is cast
        # once per forward instead of once per iteration (and its gradient
        # accumulates over the 12 iterations before a single cast back).
        gru_ops.begin_forward()
        if gpu and not torch.jit.is_tracing():
            # packed encoder-conv weights after an optimizer step: one batched
            # repack on the main stream, before any stream forks (ops/wpack.py);
            # not while tracing for export (stock ops only, nothing packed)
            wpack.refresh()
        # The context encoder (batch B) and the feature encoder + correlation
        # volume (batch 2B) are independent until the update loop: run cnet on
        # a second HIP stream so its small kernels (norm finalize, bias, ReLU
        # tails) fill the gaps of the fnet chain.  Autograd replays each
        # backward op on its forward op's stream, so the two encoder backward
        # passes overlap the same way (the engine inserts the cross-stream
        # waits).  Under hipGraph capture the fork/join becomes two parallel
        # branches of the inference graph.
        side = None
        dparams = None
        enc_defer = contextlib.nullcontext()
        if (gpu and self.cfg.overlap_encoders and OVERLAP["defer"] and self.training and torch.is_grad_enabled()
                and FusedTrainEngine.config_capable(self.cfg) and not test_mode):
            # update-block weight gradients overlap the encoder backward, and the
            # encoder convs' weight gradients overlap their own dgrad chain
            # (see DeferGrads; ops/enc_conv.py defer_weights)
            uparams = self._train_engine().params
            eparams = self._encoder_conv_params() if OVERLAP["defer_enc"] else []
            views = DeferGrads.apply(self._side_stream(dev, 1), *uparams, *eparams)
            dparams = views[:len(uparams)]
            enc_defer = enc_conv.defer_weights(self._side_stream(dev, 1),
                                               {id(p): v for p, v in zip(eparams, views[len(uparams):])})
        # (not while tracing for TorchScript export: a stream hand-off is a
        # Python autograd Function the exported graph cannot hold)
        if gpu and self.cfg.overlap_encoders and OVERLAP["cnet"] and not torch.jit.is_tracing():
            side = self._side_stream(dev)
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
        with self._autocast(dev), enc_defer:
            fused_enc = (xin is not None and self.training and not test_mode and FusedEncoders.eligible(self, xin))
            if fused_enc:
                # both encoders, forward and backward, as one scheduled node
                # (models/fused_encoder.py): fnet on main, cnet on the side stream
                xf, cnet = self._encoder_engine().run(xin, image1, side)
                fmap1, fmap2 = _SplitPair.apply(xf, image1.shape[0])
            elif side is not None:
                # fnet (main) and cnet (side) stage by stage, interleaved on the host
                xf = xin if xin is not None else torch.cat([image1, image2], dim=0)
                xc = image1
                ff, fc = self.fnet.stage_fns(), self.cnet.stage_fns()
                for k in range(max(len(ff), len(fc))):
                    if k < len(ff):
                        xf = ff[k](xf)
                    if k < len(fc):
                        with torch.cuda.stream(side):
                            xc = fc[k](xc)
                cnet = xc
                image1.record_stream(side)  # main-stream block read on side (kept by cnet's backward)
                fmap1, fmap2 = _SplitPair.apply(xf, image1.shape[0])
            else:
                fmap1, fmap2 = self.fnet([image1, image2])
            # The reference casts the features to fp32 (core/raft.py:102-103).
            # Under bf16 autocast they are exactly representable in bf16, so the
            # MFMA volume kernel consumes them in bf16 with fp32 accumulation
            # (exact products); in fp32 mode it runs the exact fp32 MFMA variant.
            if not (mixed and _ext.use_hip(fmap1)):
                fmap1, fmap2 = fmap1.float(), fmap2.float()
            corr_dtype = torch.bfloat16 if mixed else torch.float32
            block = AlternateCorrBlock if self.cfg.alternate_corr else CorrBlock
            kw = {} if self.cfg.alternate_corr else dict(pyr_dtype=self.cfg.pyr_dtype)
            corr_fn = block(fmap1, fmap2, num_levels=self.cfg.corr_levels,
                            radius=self.cfg.corr_radius, out_dtype=corr_dtype, **kw)

            if side is not None:
                main.wait_stream(side)
                cnet = _StreamHandoff.apply(cnet, side)
            elif not fused_enc:
                cnet = self.cnet(image1)
            fused_train = not test_mode and FusedTrainEngine.eligible(self, image1, corr_fn)
            fused_inf = not fused_train and FusedUpdate.eligible(self, image1, corr_fn)
            if (fused_train and not self.cfg.small) or fused_inf:
                # the fused engines split the context features and apply tanh / relu
                # themselves, straight into their buffers (context_act)
                net, inp = cnet, None
            else:
                net, inp = torch.split(cnet, [hdim, cdim], dim=1)
                net = torch.tanh(net)
                inp = torch.relu(inp)

            coords0, coords1 = self.initialize_flow(image1)
            if flow_init is not None:
                coords1 = coords1 + flow_init

            if fused_train:
                eng = self._train_engine()
                cstate, ctoken, otf_t = FusedTrainEngine.corr_inputs(corr_fn)
                otf = None if not otf_t else (corr_fn.radius, corr_fn.scale, len(otf_t) - 1)
                up = FusedTrainLoop.apply(eng, cstate, ctoken, net, inp, coords0, coords1,
                                          iters, dparams is not None, otf, *otf_t,
                                          *(dparams if dparams is not None else eng.params))
                # consecutive views of one tensor: the fused loss reads it whole
                return list(up.view(iters, *coords1.shape[:1], *up.shape[1:]).unbind(0))

            eng_t = self.__dict__.get("_fused_train")
            if (eng_t is not None and eng_t.grad_group is not None and not test_mode and self.training
                    and torch.is_grad_enabled()):
                # DDP ignores the update-block parameters: only the fused engine reduces them
                raise RuntimeError("data-parallel RAFT was wrapped for the fused training engine, "
                                   "but this step is not eligible for it (update-block gradients "
                                   "would not be all-reduced)")

            if fused_inf:
                eng = self._fused_engine()
                coords1, preds, flow_up = eng.run(net, inp, corr_fn, coords0, coords1, iters, test_mode)
                if test_mode:
                    return coords1 - coords0, flow_up
                return preds

            small = self.cfg.small
            preds = []
            flow_up = None
            for itr in range(iters):
                coords1 = coords1.detach()
                corr = corr_fn(coords1)
                flow = coords1 - coords0
                last = itr == iters - 1
                want_up = (not test_mode) or last
                if small:
                    net, up_mask, delta_flow = self.update_block(net, inp, corr, flow)
                else:
                    net, up_mask, delta_flow = self.update_block(net, inp, corr, flow,
                                                                 upsample=want_up)
                coords1 = coords1 + delta_flow.float()
                if not want_up:
                    continue
                if up_mask is None:
                    flow_up = upflow8(coords1 - coords0)
                else:
                    flow_up = self.upsample_flow(coords1 - coords0, up_mask)
                preds.append(flow_up)

        if test_mode:
            return coords1 - coords0, flow_up
        return preds
