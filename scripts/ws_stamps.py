#!/usr/bin/env python
"""Summarise conv_ws in-kernel stamps (scripts/pmc_ws.py --stamps, RS_WS_STAMPS build):
per-phase cycle medians over waves.  python scripts/ws_stamps.py FILE.npy"""
import sys

import numpy as np

st = np.load(sys.argv[1]).reshape(-1, 66).astype(np.int64)
st = st[st[:, 0] > 0]
t0 = st[:, 0].min()
print(f"waves {len(st)}  kernel span {st.max() - t0} cycles")
print(f"entry skew (max-min start) {st[:, 0].max() - t0}")
print(f"prologue (s1-s0) median {np.median(st[:, 1] - st[:, 0]):.0f}  max {np.max(st[:, 1] - st[:, 0])}")
for t in range(16):
    c = st[:, 2 + 4 * t: 5 + 4 * t]
    ok = (c > 0).all(1)
    if not ok.any():
        break
    c = c[ok]
    mf = c[:, 1] - c[:, 0]
    w1 = c[:, 2] - c[:, 1]
    nxt = st[ok, 2 + 4 * (t + 1)] - c[:, 2] if t < 15 else np.zeros(len(c))
    nxt = nxt[nxt > 0] if (nxt > 0).any() else np.array([0])
    print(f"tile {t:2d}: waves {ok.sum():5d}  mfma-phase {np.median(mf):6.0f}  partials+wait+barrier {np.median(w1):6.0f}  "
          f"to next tile {np.median(nxt):6.0f}   (mfma max {mf.max()}, wait max {w1.max()})")
