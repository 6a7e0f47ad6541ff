"""Optimizer + LR schedule (reference train.py:79-86).

AdamW(lr, weight_decay=wdecay, eps=epsilon) and a linear OneCycle schedule over
num_steps + 100 with pct_start 0.05 and no momentum cycling.

On GPU the update is :class:`FusedClipAdamW`: gradient clipping (reference
train.py:176, ``clip_grad_norm_``) and the AdamW update of all ~120 parameter
tensors in two native launches (csrc/optim.hip), the moments in two flat
buffers.  Elsewhere (CPU, ``RS_FUSED_ADAMW=0``) it is torch.optim.AdamW
(fused / foreach multi-tensor kernels where available).
"""
from __future__ import annotations

import os

import torch
import torch.optim as optim

from ..runtime import weights

_FUSED_ADAMW = os.environ.get("RS_FUSED_ADAMW", "1") != "0"


class FusedClipAdamW(optim.Optimizer):
    """torch.optim.AdamW semantics (decoupled weight decay, bias-corrected
    moments) over ONE parameter group, executed by
    ``torch.ops.raft_stir.clip_adamw_``:

    * :meth:`clip_and_step` (max_norm) = ``clip_grad_norm_(params, max_norm)``
      followed by ``step()``, in two launches; returns the total gradient norm
      (a device tensor; the ``.grad`` tensors are left unclipped);
    * :meth:`step` = the AdamW update alone (no clipping);
    * a non-finite gradient norm skips the update on the device (parameters,
      moments and the step count unchanged), as the trainer's fused-AdamW
      ``found_inf`` path does;
    * ``exp_avg`` / ``exp_avg_sq`` live in two flat fp32 buffers; the per-
      parameter state entries are views of them (parameter strides), so
      ``state_dict()`` / ``load_state_dict()`` keep torch's AdamW layout and
      checkpoints move freely between the two implementations;
    * a tensor ``lr`` (``capturable=True``) is read on the device, so the step
      can be captured in a hipGraph while the scheduler writes the lr in place.
    """

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, capturable=False):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, capturable=capturable,
                        fused=True, amsgrad=False, maximize=False, foreach=None, differentiable=False)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedClipAdamW supports one parameter group")
        ps = self.param_groups[0]["params"]
        if not ps or any(not p.is_cuda or p.dtype != torch.float32 for p in ps):
            raise ValueError("FusedClipAdamW needs fp32 parameters on the GPU")
        dev = ps[0].device
        self._moff, n = [], 0
        for p in ps:
            self._moff.append(n)
            n += p.numel()
        self._m = torch.zeros(n, device=dev, dtype=torch.float32)
        self._v = torch.zeros(n, device=dev, dtype=torch.float32)
        chunk = 8192  # csrc/optim.h CH
        self._partial = torch.empty(sum(-(-p.numel() // chunk) for p in ps) + 1, device=dev, dtype=torch.float32)
        self._state = torch.zeros(2, device=dev, dtype=torch.float32)  # (completed steps, pending flag)
        for p, o in zip(ps, self._moff):
            self._bind(p, o)

    def _bind(self, p, o):
        st = self.state[p]
        st["exp_avg"] = self._m[o:o + p.numel()].as_strided(p.shape, p.stride())
        st["exp_avg_sq"] = self._v[o:o + p.numel()].as_strided(p.shape, p.stride())
        st["step"] = self._state[0:1].view(())  # shared device step counter (see state_dict)

    @torch.no_grad()
    def _run(self, max_norm):
        from ..ops import _ext
        _ext.load(raise_on_error=True)
        g = self.param_groups[0]
        params, grads, moff = [], [], []
        for p, o in zip(g["params"], self._moff):
            gr = p.grad
            if gr is None:
                continue
            if gr.dtype != torch.float32 or gr.stride() != p.stride():
                gr = torch.empty_like(p).copy_(gr)
            params.append(p)
            grads.append(gr)
            moff.append(o)
        if not params:
            return torch.zeros((), device=self._m.device)
        lr = g["lr"]
        lr_t = lr if isinstance(lr, torch.Tensor) else None
        b1, b2 = g["betas"]
        norm = torch.ops.raft_stir.clip_adamw_(params, grads, self._m, self._v, self._partial, moff, lr_t,
                                               0.0 if lr_t is not None else float(lr), b1, b2, g["eps"],
                                               g["weight_decay"], float(max_norm), self._state)
        # the parameters changed behind autograd's back (a custom mutable op
        # bumps no _version): advance the weight generation here as well as in
        # the global step post-hook, so every packed-weight cache (ops/wpack.py,
        # the fused engines) re-packs even for a direct _run
        weights.bump()
        return norm

    def clip_and_step(self, max_norm: float):
        """Clip + update through the hooked :meth:`step` (step pre/post hooks,
        the LR scheduler's step-order bookkeeping); returns the total norm."""
        self._clip = float(max_norm)
        try:
            self.step()
        finally:
            self._clip = 0.0
        return self._last_norm

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._last_norm = self._run(getattr(self, "_clip", 0.0))
        return loss

    def state_dict(self):
        sd = super().state_dict()
        steps = float(self._state[0] + self._state[1])
        for st in sd["state"].values():
            st["step"] = torch.tensor(steps)
            st["exp_avg"] = st["exp_avg"].clone()
            st["exp_avg_sq"] = st["exp_avg_sq"].clone()
        return sd

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        ps = self.param_groups[0]["params"]
        steps = 0.0
        with torch.no_grad():
            for p, o in zip(ps, self._moff):
                st = self.state.get(p, {})
                m, v = st.get("exp_avg"), st.get("exp_avg_sq")
                if "step" in st:
                    steps = float(st["step"])
                self._bind(p, o)
                if m is not None:
                    self.state[p]["exp_avg"].copy_(m)
                    self.state[p]["exp_avg_sq"].copy_(v)
            self._state.copy_(torch.tensor([steps, 0.0]))


def fetch_optimizer(args, model, fused=None, capturable=False):
    """``capturable``: the learning rate lives in a device tensor (updated in
    place by the scheduler) and the update reads no host state, so the whole
    step can be replayed from a hipGraph (runtime/graph.py GraphedTrainStep)."""
    params = [p for p in model.parameters() if p.requires_grad]
    if fused is None:
        fused = bool(params) and params[0].is_cuda
    kw = dict(lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon)
    if capturable:
        kw.update(lr=torch.tensor(float(args.lr), device=params[0].device), capturable=True)
    optimizer = None
    if fused and _FUSED_ADAMW and all(p.is_cuda and p.dtype == torch.float32 for p in params):
        from ..ops import _ext
        if _ext.load():
            optimizer = FusedClipAdamW(params, **kw)
    if optimizer is None:
        try:
            optimizer = optim.AdamW(params, fused=fused, **kw)
        except (RuntimeError, TypeError):
            optimizer = optim.AdamW(params, foreach=fused, **kw)
    scheduler = optim.lr_scheduler.OneCycleLR(
        optimizer, args.lr, args.num_steps + 100, pct_start=0.05, cycle_momentum=False,
        anneal_strategy="linear")
    return optimizer, scheduler


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)
