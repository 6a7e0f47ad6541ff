#!/usr/bin/env python
"""Host cost of the encoders' training forward (the bench step's first phase):
enqueue time of fnet(2B images) + cnet(B images) per call without syncs, and a
cProfile of the Python side sorted by self time.

    python scripts/enc_host_profile.py
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from raft_stir_amd.config import make_args
    from raft_stir_amd.models import RAFT
    dev = torch.device("cuda", 0)
    m = RAFT(make_args(mixed_precision=True)).to(dev).to(memory_format=torch.channels_last).train()
    x2 = torch.randn(16, 3, 368, 496, device=dev).contiguous(memory_format=torch.channels_last)
    x1 = x2[:8]

    def fwd():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            a = m.fnet(x2)
            b = m.cnet(x1)
        return a, b
    for _ in range(3):
        a, b = fwd()
        (a.float().mean() + b.float().mean()).backward()
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a, b = fwd()
        ts.append(time.perf_counter() - t0)
        torch.cuda.synchronize()
    g0 = torch.cuda.Event(enable_timing=True)
    g1 = torch.cuda.Event(enable_timing=True)
    g0.record()
    for _ in range(10):
        fwd()
    g1.record()
    torch.cuda.synchronize()
    print(f"encoders fwd: host enqueue {1e3 * min(ts):.2f} ms (min of 10), GPU {g0.elapsed_time(g1) / 10:.2f} ms per call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        fwd()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
