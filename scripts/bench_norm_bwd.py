"""Time torch.ops.raft_stir.norm_act_backward alone (graph-free, cuda events)
at the fnet 1/2-res shape: 16 x 184 x 248 x 64 bf16 instance norm with a plain
residual and a second upstream gradient (a residual block's output norm), and
without them (its first norm).  Run once per RS_NORM_GSTAGE setting."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_stir_amd.ops import _ext  # noqa: E402

_ext.load(raise_on_error=True)

dev = "cuda"
B, H, W, C = 16, 184, 248, 64
g = torch.Generator(device=dev).manual_seed(0)
mk = lambda: torch.randn(B, H, W, C, device=dev, generator=g).to(torch.bfloat16)
x, dy, dy2, res = mk(), mk(), mk(), mk().relu()
mean, rstd = torch.ops.raft_stir.norm_stats(x, True, 1e-5)
gamma = torch.ones(C, device=dev)
beta = torch.zeros(C, device=dev)
R = torch.ops.raft_stir
R.norm_set_reduce_blocks(int(os.environ.get("RS_NORM_REDUCE_BLOCKS", "512")))
tag = " ".join(f"{k}={os.environ[k]}" for k in ("RS_NORM_GSTAGE", "RS_NORM_STATS_BLOCKS") if k in os.environ)
f = lambda: R.norm_stats(x, True, 1e-5)
for _ in range(5):
    f()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    f()
e1.record()
torch.cuda.synchronize()
print(f"{tag} stats: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us/call")
for name, args in (("res+dy2", (res, True, True, dy2)), ("relu only", (None, True, True, None))):
    f = lambda: R.norm_act_backward(dy, x, mean, rstd, gamma, beta, *args)
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f()
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag} {name}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us/call")
