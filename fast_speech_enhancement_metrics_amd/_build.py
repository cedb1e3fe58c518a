"""Build libfsem.so (the gfx950 HIP engine) in-tree with hipcc.

    python -m fast_speech_enhancement_metrics_amd._build

Output: fast_speech_enhancement_metrics_amd/lib/libfsem.so (git-ignored, travels with the
repo snapshot to the GPU box).  Cross-compiles without a GPU.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libfsem.so")
STAMP_LIB = os.path.join(LIBDIR, "libfsem_stamps.so")  # diagnostic build (tools/stamps.py)
SOURCES = ["pesq.hip", "stoi.hip", "resample.hip"]
HEADERS = ["fsem_common.h", "fsem_fft.h", "fsem_internal.h", "fsem_resample.h", "fsem_tables.inc"]
ARCH = os.environ.get("FSEM_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the fsem HIP engine cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(PKG, "..", "include", "fsem.h"))
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    lib = STAMP_LIB if stamps else LIB
    if not force and not stamps and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    tmp = lib + ".tmp"
    cmd = [_hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-shared", "-fPIC",
           "-Wno-unused-result", "-o", tmp] + [os.path.join(CSRC, s) for s in SOURCES]
    if stamps:
        cmd.insert(1, "-DFSEM_STAMPS")
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--stamps" in sys.argv:
        print(build(verbose=True, stamps=True))
