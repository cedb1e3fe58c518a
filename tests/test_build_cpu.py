"""Build hygiene (CPU): the library carries the content hash of the sources, headers and flags it
was built from (fsem_build_id), staleness follows that hash -- every header the kernels include
counts (fsem_vad.h included), and so do the compile flags in _build.py -- and the host layer
refuses a library whose id differs from its tree's."""
import os
import shutil

import pytest

from fast_speech_enhancement_metrics_amd import _build, _native


def test_every_included_header_is_a_build_dependency():
    import re
    deps = {os.path.basename(d) for d in _build.deps()}
    for src in _build.SOURCES + _build.HEADERS:
        text = open(os.path.join(_build.CSRC, src)).read()
        for inc in re.findall(r'#include\s+"([^"]+)"', text):
            assert os.path.basename(inc) in deps, (src, inc)


def test_library_build_id_matches_tree():
    _build.build()
    assert not _build._stale()
    assert _build.library_build_id(_build.LIB) == _build.source_hash()
    lib = _native.load()
    assert lib.fsem_build_id().decode() == _build.source_hash()
    assert lib.fsem_version() >= 6


@pytest.fixture()
def tree_copy(tmp_path, monkeypatch):
    """A copy of csrc/ + include/ the build functions point at (nothing is compiled)."""
    csrc = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, csrc)
    inc = tmp_path / "fsem.h"
    shutil.copy(_build.HEADER_ABI, inc)
    monkeypatch.setattr(_build, "CSRC", str(csrc))
    monkeypatch.setattr(_build, "HEADER_ABI", str(inc))
    return csrc


def test_header_edit_makes_library_stale(tree_copy):
    assert not _build._stale()
    vad = tree_copy / "fsem_vad.h"
    vad.write_text(vad.read_text() + "\n// edited\n")
    assert _build._stale()


def test_header_mtime_alone_does_not_rebuild(tree_copy):
    vad = tree_copy / "fsem_vad.h"
    t = os.path.getmtime(_build.LIB) + 100
    os.utime(vad, (t, t))  # newer than the library, content unchanged
    assert not _build._stale()


def test_flag_change_makes_library_stale(monkeypatch):
    assert not _build._stale()
    flags = dict(_build.SOURCE_FLAGS)
    flags["pesq.hip"] = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
    monkeypatch.setattr(_build, "SOURCE_FLAGS", flags)
    assert _build._stale()


def test_stale_library_is_refused_without_compiler(tree_copy, monkeypatch):
    vad = tree_copy / "fsem_vad.h"
    vad.write_text(vad.read_text() + "\n// edited\n")

    def no_build(*a, **k):
        raise RuntimeError("hipcc not found")

    monkeypatch.setattr(_build, "build", no_build)
    with pytest.raises(ImportError, match="stale"):
        _native._check_build_id()


def test_stale_library_is_refused_without_opt_in(tree_copy, monkeypatch):
    """A stale library is not rebuilt at import unless FSEM_AUTOBUILD=1 (every rank of a
    multi-process job would otherwise run hipcc)."""
    vad = tree_copy / "fsem_vad.h"
    vad.write_text(vad.read_text() + "\n// edited\n")
    calls = []
    monkeypatch.setattr(_build, "build", lambda *a, **k: calls.append(1))
    monkeypatch.delenv("FSEM_AUTOBUILD", raising=False)
    with pytest.raises(ImportError, match="stale"):
        _native._check_build_id()
    assert not calls


def test_other_target_is_refused_not_rebuilt(monkeypatch):
    """A library built for another offload target is refused, never silently rebuilt for this one
    (ADVICE r5); the target is recorded apart from the content hash, which it does not enter."""
    assert _build.library_build_arch(_build.LIB) == _build.ARCH
    h = _build.source_hash()
    calls = []
    monkeypatch.setattr(_build, "build", lambda *a, **k: calls.append(1))
    monkeypatch.setattr(_build, "ARCH", "gfx942")
    monkeypatch.setenv("FSEM_AUTOBUILD", "1")
    assert _build.source_hash() == h
    with pytest.raises(ImportError, match="built for gfx950"):
        _native._check_build_id()
    assert not calls


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No HIP engine -> ImportError from the loader (no CPU fallback behind a GPU metric's back)."""
    monkeypatch.setattr(_native, "LIB_PATH", str(tmp_path / "libfsem.so"))
    monkeypatch.setattr(_native, "_lib", None)
    with pytest.raises(ImportError, match="not built"):
        _native.load()
