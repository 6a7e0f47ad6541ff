"""Probe: packed-weight caches of the encoder conv kernels follow optimizer updates."""
import copy

import torch

from raft_stir_amd.models.extractor import BasicEncoder
from raft_stir_amd.ops import enc_conv

CL = torch.channels_last
dev = torch.device("cuda")
torch.manual_seed(2)
enc = BasicEncoder(output_dim=256, norm_fn="instance").to(dev).to(memory_format=CL)
x = (torch.rand(2, 3, 96, 128, device=dev) * 2 - 1).contiguous(memory_format=CL)
opt = torch.optim.AdamW(enc.parameters(), lr=1e-2, fused=True)
for step in range(3):
    opt.zero_grad(set_to_none=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = enc(x)
    y.float().square().mean().backward()
    vers = {n: p._version for n, p in enc.named_parameters()}
    opt.step()
    vers2 = {n: p._version for n, p in enc.named_parameters()}
    print("step", step, "versions bumped:", sum(vers2[n] != vers[n] for n in vers), "/", len(vers))
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        ya = enc(x).float()
        enc_conv._GEO = False
        yb = enc(x).float()
        enc_conv._GEO = True
    print("  geo vs miopen fwd after update:", ((ya - yb).norm() / yb.norm()).item())
