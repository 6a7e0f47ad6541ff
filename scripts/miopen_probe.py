"""Time MIOpen convs of the encoder shapes with and without bias (fwd+bwd)."""
import sys
import time

import torch
import torch.nn.functional as F

dev = torch.device("cuda")
shapes = [  # N, Cin, H, W, Cout, k, stride
    (16, 3, 368, 496, 64, 7, 2),
    (16, 64, 184, 248, 64, 3, 1),
    (16, 64, 184, 248, 96, 3, 2),
    (16, 96, 92, 124, 96, 3, 1),
]
for N, Ci, H, W, Co, k, s in shapes:
    x = torch.randn(N, Ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w = (torch.randn(Co, Ci, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
    w.requires_grad_(True)
    b = torch.zeros(Co, device=dev, requires_grad=True)
    for use_b in (True, False):
        for it in range(8):
            if it == 3:
                torch.cuda.synchronize()
                t0 = time.time()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = F.conv2d(x, w, b if use_b else None, s, k // 2)
            y.float().sum().backward()
        torch.cuda.synchronize()
        print(f"{(N, Ci, H, W, Co, k, s)} bias={use_b}: {(time.time() - t0) / 5 * 1e3:.2f} ms/iter", flush=True)
