"""STIR point tracker + TorchScript / ONNX export (reference rafttoonnx.py).

``RaftPointTrack(model).forward(pointlist (1,N,2) xy, image1, image2)``
    runs RAFT for ``NUMITERS`` (12) iterations in test mode, bilinearly samples
    the full-resolution flow at the points (grid_sample, align_corners=True)
    and returns ``pointlist + flow`` (1, N, 2)  (reference rafttoonnx.py:137-154).

Export (reference rafttoonnx.py:49-118, 156-223):
  * :func:`export_torchscript` -- ``torch.jit.trace`` of the tracker, saved and
    reloaded, with a parity check against eager;
  * :func:`export_onnx` -- opset 17, input names ``pointlist/image1/image2``,
    output ``end_points`` (or the bare model with ``image1/image2 ->
    flow_low/flow_up``), legacy TorchScript-based exporter (``dynamo=False``);
    optional onnxruntime parity check at atol=rtol=1e-2 when onnxruntime is
    importable (it is not in this image: parity unpinned there).
Tracing always takes the pure-ATen composite path of every op (ops/_ext.py
``_exporting``) so the graphs contain only standard operators, whichever
device the model lives on.

:class:`PointTrackServer` is the serving path on MI355X: the whole tracker
(encoders, 12 iterations, upsampling and point sampling) captured once in a
hipGraph per input shape and replayed per request with the HIP kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

NUMITERS = 12
POINTCOUNT = 32


def sample_points(flow_up: torch.Tensor, pointlist: torch.Tensor) -> torch.Tensor:
    """flow (1,2,H,W), points (1,N,2) xy pixels -> flow at points (1,N,2)."""
    H, W = flow_up.shape[-2:]
    g = pointlist.unsqueeze(2)  # (1,N,1,2)
    gx = 2 * g[..., :1] / (W - 1) - 1
    gy = 2 * g[..., 1:] / (H - 1) - 1
    s = F.grid_sample(flow_up, torch.cat([gx, gy], dim=-1), align_corners=True)  # (1,2,N,1)
    return s.squeeze(3).permute(0, 2, 1)


class RaftPointTrack(nn.Module):
    def __init__(self, model, iters: int = NUMITERS):
        super().__init__()
        self.model = model
        self.iters = iters

    def forward(self, pointlist, image1, image2):
        _, flow_up = self.model(image1, image2, iters=self.iters, test_mode=True)
        return pointlist + sample_points(flow_up.to(pointlist.dtype), pointlist)


class _FlowOnly(nn.Module):
    def __init__(self, model, iters):
        super().__init__()
        self.model = model
        self.iters = iters

    def forward(self, image1, image2):
        return self.model(image1, image2, iters=self.iters, test_mode=True)


def _reference_mode():
    from ..ops._ext import reference_mode
    return reference_mode()


@torch.no_grad()
def export_torchscript(tracker: nn.Module, example, path: str, check: bool = True,
                       atol: float = 1e-3):
    tracker.eval()
    with _reference_mode():
        traced = torch.jit.trace(tracker, example, check_trace=False)
        traced.save(path)
        loaded = torch.jit.load(path, map_location=example[0].device)
        if check:
            want = tracker(*example)
            got = loaded(*example)
            err = (want - got).abs().max().item()
            if err > atol:
                raise AssertionError(f"TorchScript parity failed: max|diff|={err}")
    return loaded


def onnx_available() -> bool:
    try:
        import onnx  # noqa: F401
        return True
    except Exception:
        return False


@torch.no_grad()
def export_onnx(module: nn.Module, example, path: str, input_names, output_names,
                opset: int = 17, check: bool = True, tol: float = 1e-2):
    module.eval()
    with _reference_mode():
        torch.onnx.export(module, example, path, export_params=True, opset_version=opset,
                          do_constant_folding=True, input_names=list(input_names),
                          output_names=list(output_names), verbose=False, dynamo=False)
    if check:
        try:
            import onnxruntime as ort
        except Exception:
            return None  # parity unpinned: onnxruntime absent
        sess = ort.InferenceSession(path, providers=["CPUExecutionProvider"])
        feeds = {n: t.detach().cpu().numpy() for n, t in zip(input_names, example)}
        outs = sess.run(None, feeds)
        with _reference_mode():
            want = module(*example)
        want = want if isinstance(want, (tuple, list)) else (want,)
        for w, o in zip(want, outs):
            if not torch.allclose(w.cpu(), torch.from_numpy(o), atol=tol, rtol=tol):
                raise AssertionError("ONNX model not close to the PyTorch model")
    return path


def export_pointtrack(model, path_prefix="raft_pointtrackSTIR", size=(512, 640),
                      npoints=POINTCOUNT, device=None, onnx=True, iters=NUMITERS):
    """Export the STIR tracker like reference convertmodelpointtrack:
    ``<prefix>.pt`` (TorchScript) and ``<prefix>.onnx`` (when onnx exists)."""
    device = device or next(model.parameters()).device
    tracker = RaftPointTrack(model, iters=iters).to(device).eval()
    H, W = size
    g = torch.Generator().manual_seed(0)
    image1 = (torch.rand(1, 3, H, W, generator=g) * 255).to(device)
    image2 = (torch.rand(1, 3, H, W, generator=g) * 255).to(device)
    points = (torch.rand(1, npoints, 2, generator=g) * min(H, W)).to(device)
    example = (points, image1, image2)
    out = {"torchscript": path_prefix + ".pt"}
    export_torchscript(tracker, example, out["torchscript"])
    if onnx and onnx_available():
        export_onnx(tracker, example, path_prefix + ".onnx", ["pointlist", "image1", "image2"],
                    ["end_points"])
        out["onnx"] = path_prefix + ".onnx"
    return out


class PointTrackServer:
    """Graphed STIR point tracker for serving on the GPU (HIP kernels)."""

    def __init__(self, model, iters: int = NUMITERS):
        self.model = model.eval()
        self.iters = iters
        self.graphs = {}

    @torch.no_grad()
    def __call__(self, pointlist, image1, image2):
        dev = next(self.model.parameters()).device
        if dev.type != "cuda":
            return RaftPointTrack(self.model, self.iters)(pointlist, image1, image2)
        key = (tuple(image1.shape), tuple(pointlist.shape))
        st = self.graphs.get(key)
        if st is None:
            st = self._capture(pointlist, image1, image2)
            self.graphs[key] = st
        st["p"].copy_(pointlist)
        st["i1"].copy_(image1)
        st["i2"].copy_(image2)
        st["graph"].replay()
        return st["out"].clone()

    def _capture(self, pointlist, image1, image2):
        p = pointlist.detach().clone()
        i1 = image1.detach().clone().contiguous(memory_format=torch.channels_last)
        i2 = image2.detach().clone().contiguous(memory_format=torch.channels_last)
        tracker = RaftPointTrack(self.model, self.iters)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                tracker(p, i1, i2)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = tracker(p, i1, i2)
        return {"graph": g, "p": p, "i1": i1, "i2": i2, "out": out}
