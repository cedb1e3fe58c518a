"""CPU-side checks of the C-ABI library: it loads without a GPU, exports exactly the
symbols include/fsem.h declares, and its host-side validation / geometry logic (no kernel
launch) behaves as documented."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(REPO, "include", "fsem.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fsem_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from fast_speech_enhancement_metrics_amd import _build, _native
    _build.build()
    return _native.load()


def test_library_exports_every_declared_symbol(lib):
    from fast_speech_enhancement_metrics_amd import _native
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r" T (fsem_[a-z0-9_]+)", out))
    decl = set(declared_functions())
    assert decl, "no declarations parsed"
    assert decl <= exported, decl - exported
    assert exported <= decl, exported - decl  # no undeclared exports in the product library
    assert set(_native.SIGNATURES) == decl


def test_version_and_errors(lib):
    assert lib.fsem_version() >= 1
    assert lib.fsem_strerror(0) == b"ok"
    assert b"workspace" in lib.fsem_strerror(-2)
    assert lib.fsem_host_buffer_mapped(None) == 0  # (no runtime call for a null buffer)


@pytest.mark.parametrize("L", [160000, 48000, 40077, 5376, 511, 255, 100])
def test_pesq_frames_matches_reference_rule(lib, L):
    # PESQ.py:128-133: pad by L % 256 (sic), then torch.stft(center=False): 1 + (L' - 512) // 256
    Lp = L + L % 256
    F = 1 + (Lp - 512) // 256 if Lp >= 512 else 0
    assert lib.fsem_pesq_frames(L) == F
    assert lib.fsem_pesq_frames(160000) == 624


def test_invalid_arguments_are_rejected_without_launch(lib):
    null = None
    assert lib.fsem_pesq_wb_f32(null, null, 4, 160000, 160000, null, null, null, 0, null) == -1
    # too short (< 20 frames): the reference's unfold raises; we return FSEM_ESHORT
    p = ctypes.c_void_p(16)
    assert lib.fsem_pesq_wb_f32(p, p, 1, 4000, 4000, null, p, p, 1 << 30, null) == -4
    # workspace too small
    assert lib.fsem_pesq_wb_f32(p, p, 4, 160000, 160000, null, p, p, 16, null) == -2
    assert lib.fsem_stoi_f32(p, p, 4, 160000, 160000, null, 16000, p, p, p, 16, null) == -2
    assert lib.fsem_stoi_workspace_bytes(4, 160000, 16000) > 0
    # rows past 2^29 samples (32-bit byte offsets in the kernels): rejected before any launch
    big = (1 << 29) + 4
    assert lib.fsem_pesq_wb_f32(p, p, 1, big, big, null, p, p, 1 << 62, null) == -1
    assert lib.fsem_stoi_f32(p, p, 1, big, big, null, 16000, p, p, p, 1 << 62, null) == -1
    assert lib.fsem_pesq_stoi_f32(p, p, 1, big, big, null, p, p, p, p, 1 << 62, null) == -1
    assert lib.fsem_resample_f32(p, 1, big, big, p, big, 16000, 10000, null) == -1
    n = (1 << 28) + 1  # 8 -> 16 kHz: 2^29 + 2 output samples
    assert lib.fsem_resample_f32(p, 1, n, n, p, 1 << 30, 8000, 16000, null) == -1
    assert lib.fsem_pesq_workspace_bytes(4096, 160000) > 4096 * 2 * 624 * 49 * 4


@pytest.mark.parametrize("orig,new,n", [(16000, 10000, 160000), (8000, 16000, 12345), (16000, 10000, 3)])
def test_resample_length_matches_torchaudio_rule(lib, orig, new, n):
    import math
    from fast_speech_enhancement_metrics_amd.resample import sinc_kernel
    _, _, o, nw = sinc_kernel(orig, new)
    assert lib.fsem_resample_length(n, orig, new) == math.ceil(nw * n / o)


def test_device_kernel_constants_match_python_restatement():
    """The compile-time 16->10 kHz kernel in csrc/fsem_tables.inc equals the torchaudio formula."""
    import numpy as np
    from fast_speech_enhancement_metrics_amd.resample import sinc_kernel
    from oracle import ta
    src = open(os.path.join(REPO, "fast_speech_enhancement_metrics_amd", "csrc", "fsem_tables.inc")).read()
    m = re.search(r"kRs16k10k\[5\]\[28\] = \{(.*?)\};", src, re.S)
    vals = np.array([float(x.strip().rstrip("f")) for x in m.group(1).split(",") if x.strip()], dtype=np.float32)
    k_py = sinc_kernel(16000, 10000)[0].numpy().ravel()
    k_or = ta.sinc_resample_kernel(16000, 10000)[0].ravel()
    np.testing.assert_array_equal(vals, k_py)
    np.testing.assert_allclose(vals, k_or, rtol=0, atol=1e-7)
