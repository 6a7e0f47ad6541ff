"""Build the in-tree HIP extension ``raft_stir_amd/_C.so`` for gfx950.

Explicit hipcc build (no hipify, no JIT cache): every ``csrc/*.hip`` is
compiled with ``hipcc --offload-arch=gfx950 -O3``, ``csrc/ops.cpp`` (the
TORCH_LIBRARY registration) as host C++ against the installed PyTorch-ROCm
headers, and everything is linked into one shared object next to this file,
so it travels with the repository snapshot to the GPU box.

Usage:  python -m raft_stir_amd.build [--force] [--jobs N] [--debug] [--asan]
(--asan: CPU AddressSanitizer + UBSan build of the host data library,
``_host_asan.so``, and a run of tests/test_data_cpu.py against it.)
Incremental: objects are rebuilt when their source, ``common.h`` or the flag
set changes.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "hip")
OUT = os.path.join(PKG, "_C.so")
HOST_CSRC = os.path.join(PKG, "csrc_host")
HOST_OUT = os.path.join(PKG, "_host.so")
HOST_ASAN_OUT = os.path.join(PKG, "_host_asan.so")
ARCH = os.environ.get("RAFT_STIR_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _flags(debug: bool):
    inc, lib, abi = _torch_paths()
    common = ["-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1",
              "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    common += ["-O0", "-g"] if debug else ["-O3"]
    hip = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", f"-I{CSRC}"]
    host = common + [f"-I{p}" for p in inc] + [f"-I{CSRC}"]
    link = ["-shared", f"-L{lib}", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lc10", "-lc10_hip",
            f"-Wl,-rpath,{lib}", f"--offload-arch={ARCH}"]
    return hip, host, link


def _sources():
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip") or f.endswith(".cpp"))
    return [os.path.join(CSRC, s) for s in srcs]


def _local_includes(path: str, seen=None) -> list:
    """The csrc/ headers ``path`` includes, transitively (``#include "x"``)."""
    seen = set() if seen is None else seen
    with open(path, "rb") as f:
        for line in f.read().decode("utf-8", "replace").splitlines():
            line = line.strip()
            if line.startswith("#include") and '"' in line:
                name = line.split('"')[1]
                hdr = os.path.join(CSRC, name)
                if name not in seen and os.path.exists(hdr):
                    seen.add(name)
                    _local_includes(hdr, seen)
    return sorted(seen)


def _digest(path: str, flags) -> str:
    h = hashlib.sha1()
    h.update(json.dumps(flags).encode())
    with open(path, "rb") as f:
        h.update(f.read())
    for hdr in _local_includes(path):
        h.update(hdr.encode())
        with open(os.path.join(CSRC, hdr), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _compile(src: str, flags, verbose: bool):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    stamp = obj + ".sha1"
    dig = _digest(src, flags)
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == dig:
                return obj, False
    cmd = [_hipcc()] + flags + ["-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{res.stdout}\n{res.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return obj, True


def build(force: bool = False, jobs: int = 0, debug: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    if force:
        for f in os.listdir(BUILD):
            os.remove(os.path.join(BUILD, f))
    hip, host, link = _flags(debug)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2) // 2), 8)
    objs, rebuilt = [], False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, hip if s.endswith(".hip") else host, verbose) for s in srcs]
        for fu in futs:
            o, changed = fu.result()
            objs.append(o)
            rebuilt |= changed
    if rebuilt or not os.path.exists(OUT):
        tmp = OUT + ".tmp"
        cmd = [_hipcc()] + objs + link + ["-o", tmp]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed\n{res.stdout}\n{res.stderr}")
        os.replace(tmp, OUT)
    return OUT


SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined"]


def build_host(force: bool = False, debug: bool = False, verbose: bool = False, sanitize: bool = False) -> str:
    """Build the CPU-only data-pipeline library ``_host.so`` (g++, zlib).
    ``sanitize``: an AddressSanitizer + UBSan build, ``_host_asan.so`` (host
    code only; loaded with the sanitizer runtimes preloaded, see run_asan)."""
    inc, lib, abi = _torch_paths()
    srcs = sorted(os.path.join(HOST_CSRC, f) for f in os.listdir(HOST_CSRC) if f.endswith(".cpp"))
    flags = ["-std=c++17", "-fPIC", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-Wno-deprecated-declarations"]
    flags += SAN_FLAGS if sanitize else (["-O0", "-g"] if debug else ["-O3"])
    flags += [f"-I{p}" for p in inc]
    out_path = HOST_ASAN_OUT if sanitize else HOST_OUT
    h = hashlib.sha1(json.dumps(flags).encode())
    for s in srcs:
        with open(s, "rb") as f:
            h.update(f.read())
    stamp = os.path.join(BUILD, "_host_asan.sha1" if sanitize else "_host.sha1")
    os.makedirs(BUILD, exist_ok=True)
    if not force and os.path.exists(out_path) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == h.hexdigest():
                return out_path
    cxx = shutil.which("g++") or shutil.which("c++")
    tmp = out_path + ".tmp"
    cmd = [cxx] + flags + srcs + [f"-L{lib}", "-ltorch_cpu", "-lc10", f"-Wl,-rpath,{lib}", "-lz",
                                  "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"host build failed\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, out_path)
    with open(stamp, "w") as f:
        f.write(h.hexdigest())
    return out_path


def sanitizer_env(lib_path: str) -> dict:
    """Environment for a python process that loads the sanitized host library:
    the ASan/UBSan runtimes preloaded (the interpreter itself is not
    instrumented), leak checking off (CPython's arenas), stop at the first
    error, and RAFT_STIR_HOST_LIB pointing the loader at ``lib_path``."""
    cxx = shutil.which("g++") or shutil.which("c++")
    rt = [subprocess.run([cxx, f"-print-file-name={n}"], capture_output=True, text=True).stdout.strip()
          for n in ("libasan.so", "libubsan.so")]
    env = dict(os.environ)
    env["LD_PRELOAD"] = ":".join([r for r in rt if os.path.isabs(r)] + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))
    env["ASAN_OPTIONS"] = "detect_leaks=0:halt_on_error=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    env["RAFT_STIR_HOST_LIB"] = lib_path
    return env


def run_asan(tests=("tests/test_data_cpu.py",), extra=()) -> int:
    """Build _host_asan.so and run the host-op tests against it (CPU only)."""
    path = build_host(sanitize=True)
    root = os.path.dirname(PKG)
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *tests, *extra]
    return subprocess.call(cmd, cwd=root, env=sanitizer_env(path))


def build_all(force: bool = False, jobs: int = 0, debug: bool = False, verbose: bool = False):
    return build(force, jobs, debug, verbose), build_host(force, debug, verbose)


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--asan", action="store_true",
                    help="build the AddressSanitizer+UBSan host library and run the data tests against it")
    a = ap.parse_args(argv)
    if a.asan:
        return run_asan()
    print(build_all(force=a.force, jobs=a.jobs, debug=a.debug, verbose=a.verbose))


if __name__ == "__main__":
    sys.exit(main())
