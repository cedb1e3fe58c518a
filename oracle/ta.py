"""ORACLE / TEST INFRASTRUCTURE ONLY.

Restatement of the torchaudio 2.8.0 operators the reference's hot path calls.  torchaudio
is a third-party dependency of the reference (``poetry.lock``: torchaudio 2.8.0) that is
absent from /root/reference and from this image, so its published algorithms are
restated here:

* ``lfilter``      -- ``torchaudio.functional.lfilter`` (reference call sites
                      ``fast_se_metrics/PESQ.py:94`` and ``:111``), sequential fp32 loop in
                      ``oracle/c/lfilter_f32.c``.
* ``resample_*``   -- ``torchaudio.transforms.Resample`` with the default
                      ``sinc_interp_hann`` / width 6 / rolloff 0.99 kernel
                      (``fast_se_metrics/base.py:13,20``).
* ``spectrogram``  -- ``torchaudio.transforms.Spectrogram(power=2, center=False)``
                      (``fast_se_metrics/PESQ.py:63-71``) = |rFFT(frame * window)|^2.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_BUILD = os.path.join(_HERE, "_build")
_LIB = os.path.join(_BUILD, "liboracle_lfilter.so")
_lib = None


def build_c(force: bool = False) -> str:
    """Compile the oracle's C restatement (gcc); output under oracle/_build/."""
    os.makedirs(_BUILD, exist_ok=True)
    src = os.path.join(_HERE, "c", "lfilter_f32.c")
    if force or not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(
            ["gcc", "-O2", "-fPIC", "-shared", "-ffp-contract=off", "-o", _LIB, src]
        )
    return _LIB


def _load():
    global _lib
    if _lib is None:
        build_c()
        lib = ctypes.CDLL(_LIB)
        fp = ctypes.POINTER(ctypes.c_float)
        lib.oracle_lfilter_f32.argtypes = [fp, fp, ctypes.c_int64, ctypes.c_int64, fp, fp, ctypes.c_int]
        lib.oracle_lfilter_f32.restype = ctypes.c_int
        lib.oracle_lfilter_iir_f32.argtypes = [fp, fp, ctypes.c_int64, ctypes.c_int64, fp, ctypes.c_int]
        lib.oracle_lfilter_iir_f32.restype = ctypes.c_int
        _lib = lib
    return _lib


def _fptr(arr: np.ndarray):
    return arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def lfilter(x: np.ndarray, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """torchaudio.functional.lfilter(x, a, b, clamp=False) on a [rows, n] float32 array."""
    lib = _load()
    x = np.ascontiguousarray(np.atleast_2d(x), dtype=np.float32)
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape
    y = np.empty_like(x)
    rc = lib.oracle_lfilter_f32(_fptr(x), _fptr(y), x.shape[0], x.shape[1], _fptr(a), _fptr(b), a.shape[0])
    if rc != 0:
        raise RuntimeError(f"oracle lfilter failed ({rc})")
    return y


def lfilter_iir(w: np.ndarray, a: np.ndarray) -> np.ndarray:
    """IIR part of torchaudio's lfilter on an already FIR-filtered float32 input."""
    lib = _load()
    w = np.ascontiguousarray(np.atleast_2d(w), dtype=np.float32)
    a = np.asarray(a, dtype=np.float32)
    a_flip = np.ascontiguousarray((a[::-1] / a[0]).astype(np.float32))
    y = np.empty_like(w)
    rc = lib.oracle_lfilter_iir_f32(_fptr(w), _fptr(y), w.shape[0], w.shape[1], _fptr(a_flip), a.shape[0])
    if rc != 0:
        raise RuntimeError(f"oracle lfilter failed ({rc})")
    return y


# ----------------------------------------------------------------------------- resample
def sinc_resample_kernel(orig_freq: int, new_freq: int, lowpass_filter_width: int = 6,
                         rolloff: float = 0.99):
    """torchaudio 2.8 ``_get_sinc_resample_kernel`` (sinc_interp_hann, dtype=None).

    Returns (kernel [new, taps] float32, width, orig_red, new_red).  Mirrors the dtype
    quirk of the original: the phase offsets ``arange(0, -new, -1) / new`` are computed in
    float32 (integer arange divided -> default dtype) before promotion to float64.
    """
    gcd = math.gcd(int(orig_freq), int(new_freq))
    orig = int(orig_freq) // gcd
    new = int(new_freq) // gcd
    base_freq = min(orig, new) * rolloff
    width = math.ceil(lowpass_filter_width * orig / base_freq)
    idx = np.arange(-width, width + orig, dtype=np.float64)[None, :] / orig
    phase = (np.arange(0, -new, -1, dtype=np.int64).astype(np.float32) / np.float32(new)).astype(np.float32)
    t = phase.astype(np.float64)[:, None] + idx
    t = t * base_freq
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    scale = base_freq / orig
    with np.errstate(invalid="ignore", divide="ignore"):
        kern = np.where(t == 0, 1.0, np.sin(t) / t)
    kern = kern * window * scale
    return kern.astype(np.float32), width, orig, new


def resample(x: np.ndarray, orig_freq: int, new_freq: int) -> np.ndarray:
    """torchaudio.transforms.Resample(orig, new)(x) for a [rows, n] float32 array.

    ``_apply_sinc_resample_kernel``: pad (width, width + orig), strided conv1d with the
    [new, 1, taps] kernel, interleave phases, truncate to ceil(new * n / orig).
    Accumulated in float64 and rounded once (conv1d order is a oneDNN detail).
    """
    x = np.atleast_2d(np.asarray(x, dtype=np.float32))
    if orig_freq == new_freq:
        return x
    kern, width, orig, new = sinc_resample_kernel(orig_freq, new_freq)
    rows, n = x.shape
    taps = kern.shape[1]
    xp = np.zeros((rows, n + 2 * width + orig), dtype=np.float64)
    xp[:, width:width + n] = x
    n_out_blocks = (xp.shape[1] - taps) // orig + 1
    # frames[r, m, t] = xp[r, orig*m + t]
    idx = orig * np.arange(n_out_blocks)[:, None] + np.arange(taps)[None, :]
    out = np.empty((rows, n_out_blocks * new), dtype=np.float32)
    k64 = kern.astype(np.float64)
    for r in range(rows):
        fr = xp[r][idx]                       # [blocks, taps]
        res = fr @ k64.T                      # [blocks, new]
        out[r] = res.reshape(-1).astype(np.float32)
    target = int(math.ceil(new * n / orig))
    return out[:, :target]


# ----------------------------------------------------------------------------- spectrogram
def hann_periodic(n: int) -> np.ndarray:
    """torch.hann_window(n) (periodic=True) in float32."""
    k = np.arange(n, dtype=np.float64)
    return (0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)).astype(np.float32)


def power_spectrogram(x: np.ndarray, n_fft: int, hop: int, window: np.ndarray) -> np.ndarray:
    """|STFT|^2, center=False, onesided, window zero-padded centred to n_fft.

    Returns [rows, frames, n_fft//2 + 1] float64 (torch.stft layout swapped to
    frame-major).
    """
    x = np.atleast_2d(np.asarray(x, dtype=np.float32))
    rows, n = x.shape
    win = np.zeros(n_fft, dtype=np.float64)
    off = (n_fft - window.shape[0]) // 2
    win[off:off + window.shape[0]] = window
    nfr = 1 + (n - n_fft) // hop
    if nfr <= 0:
        return np.zeros((rows, 0, n_fft // 2 + 1))
    idx = hop * np.arange(nfr)[:, None] + np.arange(n_fft)[None, :]
    out = np.empty((rows, nfr, n_fft // 2 + 1), dtype=np.float64)
    for r in range(rows):
        fr = x[r].astype(np.float64)[idx] * win[None, :]
        spec = np.fft.rfft(fr, axis=1)
        out[r] = spec.real ** 2 + spec.imag ** 2
    return out
