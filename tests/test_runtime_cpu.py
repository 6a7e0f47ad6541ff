"""runtime/profiler.py on a CPU-only host."""
import os
import time

import torch

from raft_stir_amd.runtime.profiler import PhaseTimer, trace


def test_phase_timer_cpu():
    pt = PhaseTimer()
    for _ in range(2):
        with pt("a"):
            time.sleep(0.01)
        with pt("b"):
            pass
    s = pt.summary()
    assert set(s) == {"a", "b"}
    assert 5 < s["a"] < 500 and s["b"] < s["a"]
    assert pt.summary() == {}          # reset
    off = PhaseTimer(enabled=False)
    with off("x"):
        pass
    assert off.summary() == {}


def test_trace_writes_files(tmp_path):
    d = str(tmp_path / "tr")
    with trace(d):
        torch.randn(32, 32) @ torch.randn(32, 32)
    assert os.path.getsize(os.path.join(d, "trace.json")) > 0
    assert "aten::mm" in open(os.path.join(d, "ops.txt")).read()
