"""Training runtime on CPU: the full train() loop (synthetic stage), reference
checkpoint names, exact resume after an injected fault, non-finite skipping,
optimizer/schedule parity with the reference hyper-parameters."""
import os

import pytest
import torch

from raft_stir_amd.train import checkpoint as ckpt
from raft_stir_amd.train import trainer

BASE = ["--device", "cpu", "--stage", "synthetic", "--small", "--iters", "2", "--image_size", "128", "128",
        "--batch_size", "2", "--num_workers", "0", "--lr", "0.0004", "--wdecay", "0.0001",
        "--synthetic_length", "6", "--sum_freq", "2", "--val_freq", "3"]


def _run(tmp_path, name, extra):
    argv = BASE + ["--name", name, "--ckpt_dir", str(tmp_path / "ck"), "--log_dir", str(tmp_path / "logs")] + extra
    return trainer.main(argv)


def test_train_loop_checkpoints_and_logs(tmp_path):
    path = _run(tmp_path, "t1", ["--num_steps", "4"])
    ck = tmp_path / "ck"
    assert os.path.exists(path) and (ck / "3_t1.pth").exists() and (ck / "t1_resume_3.pt").exists()
    sd = torch.load(path, weights_only=True)
    assert all(k.startswith("module.") for k in sd) and len(sd) == 106
    lines = open(tmp_path / "logs" / "metrics.jsonl").read().strip().splitlines()
    assert lines and '"epe"' in lines[0] and '"pairs_per_s"' in lines[0]


def test_resume_after_fault_is_exact(tmp_path):
    ref_path = _run(tmp_path / "a", "run", ["--num_steps", "5"])
    with pytest.raises(trainer.InjectedFault):
        _run(tmp_path / "b", "run", ["--num_steps", "5", "--fault_at_step", "4"])
    assert ckpt.latest_resume(str(tmp_path / "b" / "ck"), "run").endswith("run_resume_3.pt")
    res_path = _run(tmp_path / "b", "run", ["--num_steps", "5", "--resume", "auto"])
    a = torch.load(ref_path, weights_only=True)
    b = torch.load(res_path, weights_only=True)
    for k in a:
        torch.testing.assert_close(b[k], a[k], atol=0, rtol=0, msg=k)


def test_resume_with_noise_is_exact(tmp_path):
    """--add_noise draws from its own generator: its state (and every rank's
    RNG) lives in the per-rank sidecar, so a resumed run continues the noise
    stream instead of restarting it from the seed."""
    extra = ["--num_steps", "5", "--add_noise"]
    ref_path = _run(tmp_path / "a", "nz", extra)
    with pytest.raises(trainer.InjectedFault):
        _run(tmp_path / "b", "nz", extra + ["--fault_at_step", "4"])
    assert os.path.exists(ckpt.rank_rng_path(str(tmp_path / "b" / "ck" / "nz_resume_3.pt"), 0))
    res_path = _run(tmp_path / "b", "nz", extra + ["--resume", "auto"])
    a = torch.load(ref_path, weights_only=True)
    b = torch.load(res_path, weights_only=True)
    for k in a:
        torch.testing.assert_close(b[k], a[k], atol=0, rtol=0, msg=k)


def test_rank_rng_sidecar_roundtrip(tmp_path):
    p = str(tmp_path / "r_resume_1.pt")
    g = torch.Generator().manual_seed(5)
    torch.manual_seed(11)
    ckpt.save_rank_rng(p, 3, {"noise": g})
    want_t, want_g = torch.rand(4), torch.rand(4, generator=g)
    torch.manual_seed(99)
    g2 = torch.Generator().manual_seed(0)
    assert ckpt.load_rank_rng(p, 3, {"noise": g2})
    torch.testing.assert_close(torch.rand(4), want_t, atol=0, rtol=0)
    torch.testing.assert_close(torch.rand(4, generator=g2), want_g, atol=0, rtol=0)
    assert not ckpt.load_rank_rng(p, 4)


def test_resume_file_contents(tmp_path):
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.optim import fetch_optimizer
    import argparse
    m = RAFT(make_args(small=True))
    opt, sch = fetch_optimizer(argparse.Namespace(lr=1e-3, wdecay=1e-4, epsilon=1e-8, num_steps=50), m)
    for _ in range(3):
        opt.zero_grad()
        sum(p.sum() for p in m.parameters()).backward()
        opt.step()
        sch.step()
    p = str(tmp_path / "x_resume_3.pt")
    ckpt.save_resume(p, m, opt, sch, step=3, extra={"epoch": 1, "batch": 2})
    m2 = RAFT(make_args(small=True))
    opt2, sch2 = fetch_optimizer(argparse.Namespace(lr=1e-3, wdecay=1e-4, epsilon=1e-8, num_steps=50), m2)
    obj = ckpt.load_resume(p, m2, opt2, sch2)
    assert obj["step"] == 3 and obj["extra"] == {"epoch": 1, "batch": 2}
    assert sch2.get_last_lr() == sch.get_last_lr()
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_onecycle_matches_reference_schedule():
    import argparse
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    from raft_stir_amd.train.optim import fetch_optimizer
    m = RAFT(make_args(small=True))
    args = argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=1000)
    opt, sch = fetch_optimizer(args, m)
    ref_opt = torch.optim.AdamW(m.parameters(), lr=4e-4, weight_decay=1e-4, eps=1e-8)
    ref = torch.optim.lr_scheduler.OneCycleLR(ref_opt, 4e-4, 1100, pct_start=0.05,
                                              cycle_momentum=False, anneal_strategy="linear")
    for _ in range(200):
        assert abs(sch.get_last_lr()[0] - ref.get_last_lr()[0]) < 1e-12
        opt.step(); sch.step(); ref_opt.step(); ref.step()
    assert opt.param_groups[0]["weight_decay"] == 1e-4 and opt.param_groups[0]["eps"] == 1e-8


def test_nonfinite_step_skipped_on_cpu(tmp_path, monkeypatch):
    """A NaN loss must not corrupt the weights: the optimizer step is skipped."""
    from raft_stir_amd.train import loss as loss_mod
    calls = {"n": 0}
    real = loss_mod.sequence_loss

    def poisoned(*a, **k):
        l, m = real(*a, **k)
        calls["n"] += 1
        return (l * float("nan") if calls["n"] == 2 else l), m

    monkeypatch.setattr(trainer, "sequence_loss", poisoned)
    path = _run(tmp_path, "nan", ["--num_steps", "3", "--max_skips", "5"])
    sd = torch.load(path, weights_only=True)
    assert all(torch.isfinite(v).all() for v in sd.values() if v.is_floating_point())
    lines = open(tmp_path / "logs" / "metrics.jsonl").read()
    assert '"skipped": 1.0' in lines


def test_bilinear_x8_adjoint_matrices():
    """RAFT-small's fused engine differentiates the x8 align_corners upsampling
    as two GEMMs (models/fused_train.py:_interp_matrix): same forward and
    adjoint as upsample_bilinear2d."""
    import torch.nn.functional as F
    from raft_stir_amd.models.fused_train import _interp_matrix
    H, W = 13, 21
    x = torch.randn(3, 2, H, W, dtype=torch.float64).float().requires_grad_()
    up = F.interpolate(x, size=(8 * H, 8 * W), mode="bilinear", align_corners=True)
    ah, aw = _interp_matrix(H, 8 * H, "cpu"), _interp_matrix(W, 8 * W, "cpu")
    torch.testing.assert_close(ah @ x.detach() @ aw.t(), up.detach(), rtol=0, atol=2e-6)
    g = torch.randn_like(up)
    up.backward(g)
    torch.testing.assert_close(ah.t() @ g @ aw, x.grad, rtol=1e-5, atol=1e-4)


def test_deterministic_flag_plumbing():
    from raft_stir_amd.config import make_args, resolve_config
    from raft_stir_amd.train.trainer import build_parser
    assert resolve_config(make_args(deterministic=True)).deterministic
    assert not resolve_config(make_args()).deterministic
    a = build_parser().parse_args(["--deterministic"])
    assert a.deterministic


def test_fused_adamw_does_not_bump_version_but_generation_moves():
    """Why the packed-weight caches key on runtime.weights.generation(): an
    optimizer step may update parameters without bumping ``_version``
    (fused / foreach kernels); the global post-step hook always fires."""
    from raft_stir_amd.runtime import weights as wg
    p = torch.nn.Parameter(torch.randn(4))
    opt = torch.optim.SGD([p], lr=0.1, foreach=True)
    p.grad = torch.ones(4)
    g0 = wg.generation()
    opt.step()
    assert wg.generation() == g0 + 1


def test_wpack_views_never_move():
    """layouts registered after a first pack (a second model) go to
    a new chunk; the earlier views keep their storage (a captured graph reads
    them) and stay current after an update; dead models' chunks are dropped."""
    import gc
    from raft_stir_amd.ops import wpack
    from raft_stir_amd.ops.conv import pack_weight
    lay = lambda ws: pack_weight(ws[0], [(32, [(0, 32, 0)])], 64, torch.float32)
    w1 = torch.nn.Parameter(torch.randn(40, 32, 3, 3))
    a = wpack.packed(("mv1", id(w1)), [w1], lay)
    ptr = a.data_ptr()
    reg = wpack._REGS[w1.device]
    n_chunks = len(reg.chunks)
    w2 = torch.nn.Parameter(torch.randn(40, 32, 3, 3))
    b = wpack.packed(("mv2", id(w2)), [w2], lay)
    assert len(reg.chunks) == n_chunks + 1
    a2 = wpack.packed(("mv1", id(w1)), [w1], lay)
    assert a2.data_ptr() == ptr
    with torch.no_grad():
        w1.add_(1.0)
    wpack.refresh()
    assert torch.equal(a, lay([w1.detach()]).to(torch.bfloat16))
    assert torch.equal(b, lay([w2.detach()]).to(torch.bfloat16))
    del w2, b
    gc.collect()
    w3 = torch.nn.Parameter(torch.randn(40, 32, 3, 3))
    wpack.packed(("mv3", id(w3)), [w3], lay)
    assert all(c.alive() for c in reg.chunks)
    assert a.data_ptr() == ptr and torch.equal(a, lay([w1.detach()]).to(torch.bfloat16))


def test_wpack_batched_layouts_follow_updates():
    """ops/wpack.py: layouts registered as index maps into the parameters,
    all views of one flat buffer, repacked together after an optimizer step
    (which need not bump _version) and equal to the direct layout."""
    from raft_stir_amd.ops import wpack
    from raft_stir_amd.ops.conv import pack_weight, pad_to
    torch.manual_seed(0)
    w1 = torch.nn.Parameter(torch.randn(96, 64, 3, 3))
    w2 = torch.nn.Parameter(torch.randn(96, 64, 1, 1))
    lay1 = lambda ws: pack_weight(ws[0], [(64, [(0, 64, 0)])], 128, torch.float32)
    lay2 = lambda ws: pack_weight(torch.cat([ws[0][:, :, 1:2, 1:2], ws[1]], 0).transpose(0, 1),
                                  [(192, [(0, 192, 0)])], 128, torch.float32)
    for step in range(3):
        a = wpack.packed(("t1", id(w1)), [w1], lay1)
        b = wpack.packed(("t2", id(w1), id(w2)), [w1, w2], lay2)
        assert torch.equal(a, lay1([w1.detach()]).to(torch.bfloat16))
        assert torch.equal(b, lay2([w1.detach(), w2.detach()]).to(torch.bfloat16))
        w1.grad, w2.grad = torch.randn_like(w1), torch.randn_like(w2)
        torch.optim.SGD([w1, w2], lr=0.5, foreach=True).step()


def test_wpack_split_layout_matches_split_weight():
    """wpack.packed_split (gathered [wh | wl] chunks) == ops/conv.py split_weight
    of the fp32 packed layout, for a channels_last source."""
    from raft_stir_amd.ops import wpack
    from raft_stir_amd.ops.conv import pack_weight, pad_to, split_weight
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(40, 64, 3, 3).contiguous(memory_format=torch.channels_last))
    lay = lambda ws: pack_weight(ws[0], [(64, [(0, 64, 0)])], pad_to(40, 128), torch.float32)  # noqa: E731
    got = wpack.packed_split(("split_test", id(w)), [w], lay)
    want = split_weight(lay([w.detach()]))
    assert got.shape == want.shape and got.dtype == torch.bfloat16
    assert torch.equal(got, want)
