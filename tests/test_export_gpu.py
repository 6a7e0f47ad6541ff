"""TorchScript export of the STIR point tracker ON THE GPU (reference
rafttoonnx.py:133-190 convertmodelpointtrack): tracing must not record the
engine's multi-stream hand-off (a Python autograd Function) or any raft_stir
op, and the reloaded module must match the eager tracker."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pointtrack_torchscript_export_on_gpu(cuda, tmp_path):
    from raft_stir_amd.config import make_args
    from raft_stir_amd.export.pointtrack import RaftPointTrack, export_torchscript
    from raft_stir_amd.models import RAFT
    torch.manual_seed(0)
    m = RAFT(make_args(small=True)).to(cuda).eval()
    g = torch.Generator(device="cpu").manual_seed(1)
    i1 = (torch.rand(1, 3, 128, 160, generator=g) * 255).to(cuda)
    i2 = (torch.rand(1, 3, 128, 160, generator=g) * 255).to(cuda)
    pts = (torch.rand(1, 16, 2, generator=g) * 120).to(cuda)
    loaded = export_torchscript(RaftPointTrack(m, 4).eval(), (pts, i1, i2), str(tmp_path / "pt.pt"))
    graph = str(loaded.inlined_graph)
    assert "raft_stir::" not in graph and "StreamHandoff" not in graph
    with torch.no_grad():
        want = RaftPointTrack(m, 4)(pts, i1, i2)
        torch.testing.assert_close(loaded(pts, i1, i2), want, atol=2e-3, rtol=2e-3)
