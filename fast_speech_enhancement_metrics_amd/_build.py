"""Build libfsem.so (the gfx950 HIP engine) in-tree with hipcc.

    python -m fast_speech_enhancement_metrics_amd._build

Output: fast_speech_enhancement_metrics_amd/lib/libfsem.so (git-ignored, travels with the
repo snapshot to the GPU box).  Cross-compiles without a GPU.
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIBDIR, "libfsem.so")
STAMP_LIB = os.path.join(LIBDIR, "libfsem_stamps.so")  # diagnostic build (tools/stamps.py)
SOURCES = ["pesq.hip", "pesq_back.hip", "stoi.hip", "resample.hip", "align.hip"]
# per-source code-generation flags: the STOI kernels and the resamplers are scheduled for ILP
# (gfx950's max-ilp machine scheduler: joint call 7.167 vs 7.198 ms, profiles/r4_sc/; config 5
# 224.0k vs 221.3k utt/s, profiles/r4_fl/; bitwise equal); the PESQ front end keeps the
# default, under which it does not spill (max-ilp: 476 SGPR spills), and so does the time
# alignment (max-ilp: 19.68 vs 19.49 ms per 4096-row aligned PESQ step)
_ILP = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
# pesq.hip (the front end) without the SLP vectoriser (round 5): it paired scalar FMAs with literal constants
# into v_pk_fma_f32 whose constant pairs each cost two s_mov_b32 (the chunk scan: 243 of its 468
# instructions); the kernels are issue bound (every issued instruction, SALU included, costs the
# wave ~4 cycles: SQ_ACTIVE_INST_SCA / SQ_INSTS_SALU = 1 quad-cycle), and the packed forms that
# pay (FFT butterflies, pass 1's functionals, pass 2's cascade) are written out explicitly.
# Joint front end 4.478 -> 4.392 ms per 4096-row launch, profiles/r5_pk/.  The back end
# (pesq_back.hip) keeps it: its 49-band loops pack into fewer instructions with it.
SOURCE_FLAGS = {"pesq.hip": ["-fno-slp-vectorize"], "stoi.hip": _ILP, "resample.hip": _ILP}
HEADERS = ["fsem_common.h", "fsem_fft.h", "fsem_internal.h", "fsem_pesq.h", "fsem_resample.h", "fsem_tables.inc",
           "fsem_vad.h"]
HEADER_ABI = os.path.join(PKG, "..", "include", "fsem.h")
ARCH = os.environ.get("FSEM_OFFLOAD_ARCH", "gfx950")
# code-generation flags; the target (--offload-arch=ARCH) is added at build time and recorded in
# the library on its own (FSEM_BUILD_ARCH): a library built for another target is refused at
# load, never silently rebuilt (_native._check_build_id)
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wno-unused-result"]
BASE_FLAGS = FLAGS + [f"--offload-arch={ARCH}"]
_ID_MARKER = b"FSEM_BUILD_ID:"
_ARCH_MARKER = b"FSEM_BUILD_ARCH:"
# the drop-in call's list-of-dicts builder (host C, CPython API; csrc/score_list.c)
SCORE_LIST_SRC = os.path.join(CSRC, "score_list.c")
SCORE_LIST = os.path.join(LIBDIR, "_score_list" + sysconfig.get_config_var("EXT_SUFFIX"))


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the fsem HIP engine cannot be built")


def deps() -> list:
    """Every file whose content the library depends on."""
    return [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [HEADER_ABI]


def source_hash() -> str:
    """Content hash of the sources, the headers (csrc/*.h, fsem_tables.inc, include/fsem.h) and
    the code-generation flags (FLAGS, SOURCE_FLAGS; not the target, see library_build_arch): the
    library's build id (fsem_build_id())."""
    h = hashlib.sha256()
    for d in deps():
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    h.update(repr((FLAGS, sorted(SOURCE_FLAGS.items()))).encode())
    return h.hexdigest()[:16]


def library_build_id(path: str = LIB):
    """The build id embedded in a built library (read from the file, not loaded), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(_ID_MARKER) + rb"([0-9a-z]+)\0", data)
    return m.group(1).decode() if m else None


def library_build_arch(path: str = LIB):
    """The offload target a built library was compiled for (read from the file), or None."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(_ARCH_MARKER) + rb"([0-9a-z_:+-]+)\0", data)
    return m.group(1).decode() if m else None


def _stale() -> bool:
    """True when libfsem.so is missing or was built from other sources or flags than the tree's
    (content hash: an edited header or a changed SOURCE_FLAGS entry rebuilds; a touched file
    whose content is unchanged does not), or for another target than ARCH."""
    return library_build_id(LIB) != source_hash() or library_build_arch(LIB) != ARCH


def build(force: bool = False, verbose: bool = False, stamps: bool = False) -> str:
    lib = STAMP_LIB if stamps else LIB
    if not force and not stamps and not _stale():
        return LIB
    os.makedirs(LIBDIR, exist_ok=True)
    # per-process object directory and temporary library: concurrent builds do not overwrite
    # each other's objects; the finished library replaces the old one atomically
    objdir = os.path.join(LIBDIR, f"obj{'_stamps' if stamps else ''}.{os.getpid()}")
    os.makedirs(objdir, exist_ok=True)
    base = [_hipcc()] + BASE_FLAGS + [f'-DFSEM_BUILD_ID="{source_hash()}"', f'-DFSEM_BUILD_ARCH="{ARCH}"']
    if stamps:
        base.append("-DFSEM_STAMPS")
    objs = []
    try:
        procs = []
        for src in SOURCES:  # one object per source (per-source flags, compiled in parallel), one library
            obj = os.path.join(objdir, src.replace(".hip", ".o"))
            cmd = base + SOURCE_FLAGS.get(src, []) + ["-c", "-o", obj, os.path.join(CSRC, src)]
            if verbose:
                print(" ".join(cmd))
            procs.append((subprocess.Popen(cmd, cwd=CSRC), cmd))
            objs.append(obj)
        for p, cmd in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        tmp = f"{lib}.{os.getpid()}.tmp"
        cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.check_call(cmd, cwd=CSRC)
        os.replace(tmp, lib)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    return lib


def build_score_list(force: bool = False, verbose: bool = False) -> str:
    """Compile the host-side list builder (gcc, no GPU) next to libfsem.so."""
    if not force and os.path.exists(SCORE_LIST) and os.path.getmtime(SCORE_LIST) >= os.path.getmtime(SCORE_LIST_SRC):
        return SCORE_LIST
    os.makedirs(LIBDIR, exist_ok=True)
    cc = os.environ.get("CC") or shutil.which("gcc") or shutil.which("cc")
    if not cc:
        raise RuntimeError("no C compiler found: the score-list builder cannot be built")
    tmp = SCORE_LIST + f".{os.getpid()}.tmp"
    cmd = [cc, "-O2", "-shared", "-fPIC", f"-I{sysconfig.get_paths()['include']}", "-o", tmp, SCORE_LIST_SRC]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    os.replace(tmp, SCORE_LIST)
    return SCORE_LIST


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build_score_list(force="--force" in sys.argv, verbose=True))
    if "--stamps" in sys.argv:
        print(build(verbose=True, stamps=True))
