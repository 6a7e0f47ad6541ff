"""Sanitizer run of the native host code.

The data-pipeline library (raft_stir_amd/csrc_host/dataops.cpp: PNG codec,
resize, colour jitter, sparse-flow resize) parses untrusted files, so it is
rebuilt with AddressSanitizer + UndefinedBehaviorSanitizer
(``python -m raft_stir_amd.build --asan`` -> ``_host_asan.so``) and the
host-op tests -- including the corrupt/truncated-PNG cases -- run against it
in a child interpreter with the sanitizer runtimes preloaded.  Any heap
overflow, use-after-free or UB aborts that child, failing this test.
(GPU kernels are not sanitized: device ASan / XNACK is unavailable on the
MI355X pool; they are bounds-guarded and tested at ragged sizes instead.)
"""
import shutil

import pytest


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_host_ops_clean_under_asan_ubsan():
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    from raft_stir_amd.build import run_asan
    rc = run_asan(tests=("tests/test_data_cpu.py",),
                  extra=("-k", "png or resize or jitter or sparse or kitti or flo or pfm"))
    assert rc == 0, f"sanitized host-op tests failed (exit {rc})"
