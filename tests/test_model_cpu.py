"""Model-level golden tests on CPU.

* parameter counts and state_dict layout (keys, shapes, dtypes) match the
  reference (5,257,536 / 990,162 params; 179 / 106 keys);
* with identical weights our CPU forward is bit-identical to the unmodified
  reference RAFT (imported read-only from /root/reference when mounted);
* ``module.``-prefixed (DataParallel) checkpoints load; freeze_bn; flow_init;
* BASELINE config #1: RAFT-small, 4 iterations on two demo frames (CPU).
"""
import argparse
import copy
import glob
import os

import numpy as np
import pytest
import torch

from raft_stir_amd.config import make_args
from raft_stir_amd.models import RAFT
from raft_stir_amd.train import checkpoint as ckpt

DEMO = "/root/reference/demo-frames"


def _imgs(B=1, H=128, W=192, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(B, 3, H, W, generator=g) * 255, torch.rand(B, 3, H, W, generator=g) * 255


@pytest.mark.parametrize("small,params,keys", [(False, 5257536, 179), (True, 990162, 106)])
def test_param_count_and_keys(small, params, keys):
    m = RAFT(make_args(small=small))
    assert sum(p.numel() for p in m.parameters()) == params
    assert len(m.state_dict()) == keys


def test_namespace_mutation_like_reference():
    a = argparse.Namespace(small=False, mixed_precision=False)
    RAFT(a)
    assert a.corr_levels == 4 and a.corr_radius == 4 and a.dropout == 0 and a.alternate_corr is False
    b = argparse.Namespace(small=True, mixed_precision=False)
    RAFT(b)
    assert b.corr_radius == 3


@pytest.mark.parametrize("small", [False, True])
def test_state_dict_layout_matches_reference(reference_raft, small):
    torch.manual_seed(0)
    ref = reference_raft(argparse.Namespace(small=small, mixed_precision=False))
    ours = RAFT(make_args(small=small))
    rs, os_ = ref.state_dict(), ours.state_dict()
    assert list(rs.keys()) == list(os_.keys())
    for k in rs:
        assert rs[k].shape == os_[k].shape and rs[k].dtype == os_[k].dtype, k


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("alt", [False, True])
def test_forward_bitexact_vs_reference(reference_raft, small, alt):
    torch.manual_seed(0)
    ref = reference_raft(argparse.Namespace(small=small, mixed_precision=False)).eval()
    ours = RAFT(make_args(small=small, alternate_corr=alt)).eval()
    ours.load_state_dict(ref.state_dict(), strict=True)
    i1, i2 = _imgs()
    with torch.no_grad():
        a = ref(i1, i2, iters=4, test_mode=True)
        b = ours(i1, i2, iters=4, test_mode=True)
    tol = 0.0 if not alt else 1e-3  # on-the-fly corr sums in a different order
    for x, y in zip(a, b):
        assert (x - y).abs().max().item() <= tol


@pytest.mark.parametrize("small", [False, True])
def test_training_forward_matches_reference(reference_raft, small):
    torch.manual_seed(1)
    ref = reference_raft(argparse.Namespace(small=small, mixed_precision=False)).train()
    ours = RAFT(make_args(small=small)).train()
    ours.load_state_dict(ref.state_dict(), strict=True)
    i1, i2 = _imgs(B=2, seed=3)
    pa = ref(i1, i2, iters=3)
    pb = ours(i1, i2, iters=3)
    assert len(pa) == len(pb) == 3
    for x, y in zip(pa, pb):
        torch.testing.assert_close(y, x, atol=0, rtol=0)
    sum(p.abs().mean() for p in pa).backward()
    sum(p.abs().mean() for p in pb).backward()
    for (n, p), (_, q) in zip(ref.named_parameters(), ours.named_parameters()):
        torch.testing.assert_close(q.grad, p.grad, atol=1e-6, rtol=1e-4, msg=n)


def test_dataparallel_prefixed_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = RAFT(make_args(small=True))
    path = str(tmp_path / "raft-small.pth")
    ckpt.save_weights(m, path)  # reference layout: module.-prefixed fp32
    sd = torch.load(path, weights_only=True)
    assert all(k.startswith("module.") for k in sd)
    m2 = RAFT(make_args(small=True))
    res = ckpt.load_weights(m2, path, strict=True)
    assert not res.missing_keys and not res.unexpected_keys
    for (k, v), (_, w) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v, w), k
    # also loadable by plain nn.DataParallel(RAFT) like the reference tools
    dp = torch.nn.DataParallel(RAFT(make_args(small=True)))
    dp.load_state_dict(sd)


def test_freeze_bn_and_flow_init():
    torch.manual_seed(0)
    m = RAFT(make_args()).train()
    m.freeze_bn()
    bns = [x for x in m.modules() if isinstance(x, torch.nn.BatchNorm2d)]
    assert bns and all(not b.training for b in bns)
    m.eval()
    i1, i2 = _imgs()
    init = torch.randn(1, 2, 16, 24)
    with torch.no_grad():
        lo0, _ = m(i1, i2, iters=1, test_mode=True)
        lo1, _ = m(i1, i2, iters=1, flow_init=init, test_mode=True)
    assert not torch.allclose(lo0, lo1)


def test_test_mode_returns_last_prediction():
    torch.manual_seed(0)
    m = RAFT(make_args()).eval()
    i1, i2 = _imgs()
    with torch.no_grad():
        preds = m(i1, i2, iters=3, test_mode=False)
        lo, up = m(i1, i2, iters=3, test_mode=True)
    assert len(preds) == 3
    torch.testing.assert_close(up, preds[-1])
    assert lo.shape == (1, 2, 16, 24) and up.shape == (1, 2, 128, 192)


@pytest.mark.skipif(not os.path.isdir(DEMO), reason="demo frames not mounted")
def test_config1_small_4iter_demo_frames(reference_raft):
    """BASELINE config #1: RAFT-small, 4-iter forward on two demo frames, CPU."""
    from PIL import Image
    from raft_stir_amd.utils.padder import InputPadder
    files = sorted(glob.glob(os.path.join(DEMO, "*.png")))[:2]
    ims = [torch.from_numpy(np.array(Image.open(f)).astype(np.uint8)[..., :3]).permute(2, 0, 1)
           .float()[None] for f in files]
    padder = InputPadder(ims[0].shape)
    i1, i2 = padder.pad(*ims)
    torch.manual_seed(0)
    ref = reference_raft(argparse.Namespace(small=True, mixed_precision=False)).eval()
    ours = RAFT(make_args(small=True)).eval()
    ours.load_state_dict(copy.deepcopy(ref.state_dict()))
    with torch.no_grad():
        _, a = ref(i1, i2, iters=4, test_mode=True)
        _, b = ours(i1, i2, iters=4, test_mode=True)
    assert padder.unpad(b).shape[-2:] == (436, 1024)
    torch.testing.assert_close(b, a, atol=0, rtol=0)
