"""Probe: stem (7x7/s2, MIOpen) weight-gradient error vs fp32 with MIOpen's
deterministic flag on / off (tests/test_determinism_gpu.py tolerance)."""
import torch

from raft_stir_amd.models.extractor import BasicEncoder
from raft_stir_amd.runtime.determinism import deterministic

CL = torch.channels_last
dev = torch.device("cuda")
torch.manual_seed(2)
enc = BasicEncoder(output_dim=256, norm_fn="instance").to(dev).to(memory_format=CL)
x = (torch.rand(4, 3, 192, 256, device=dev) * 2 - 1).contiguous(memory_format=CL)
res = {}
for mode in ("fp32", "bf16", "bf16_det", "bf16_b", "bf16_det_b"):
    enc.zero_grad(set_to_none=True)
    with deterministic("det" in mode):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=mode != "fp32"):
            y = enc(x)
        y.float().square().mean().backward()
    torch.cuda.synchronize()
    res[mode] = {n: p.grad.detach().float().clone() for n, p in enc.named_parameters() if p.grad is not None}
rel = lambda a, b: ((a - b).norm() / b.norm()).item()
for n in ("conv1.weight", "layer1.0.conv1.weight", "layer2.0.conv1.weight", "layer2.0.downsample.0.weight",
          "conv2.weight"):
    print(n, {m: round(rel(res[m][n], res["fp32"][n]), 4) for m in res if m != "fp32"},
          "b-vs-det", round(rel(res["bf16"][n], res["bf16_det"][n]), 4))
