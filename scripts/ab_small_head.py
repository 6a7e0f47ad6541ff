#!/usr/bin/env python
"""A/B of RAFT-small's bf16 conv padding for the weight-streaming tiles
(models/fused_update.py: _SMALL_HEAD_K 128 / 96, _SMALL_Q_PAD 1 / 0):
``--k 96|128 --qpad 0|1`` then runs scripts/infer_only.py or scripts/stir_only.py in
this process with the remaining arguments.

    python scripts/ab_small_head.py --k 96 --stir -- --bf16 --reps 50
"""
import argparse
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--k", type=int, default=128)
ap.add_argument("--qpad", type=int, default=1, help="_SMALL_Q_PAD (GRU-q segments padded to 64-multiples)")
ap.add_argument("--stir", action="store_true")
a, rest = ap.parse_known_args()
from raft_stir_amd.models import fused_update  # noqa: E402
fused_update._SMALL_HEAD_K = a.k
fused_update._SMALL_Q_PAD = bool(a.qpad)
script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stir_only.py" if a.stir else "infer_only.py")
sys.argv = [script] + [x for x in rest if x != "--"]
runpy.run_path(script, run_name="__main__")
