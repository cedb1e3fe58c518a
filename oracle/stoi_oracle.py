"""ORACLE / TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's STOI / ESTOI.

Follows ``fast_se_metrics/STOI.py`` step by step (10 kHz internal rate; inputs at other
rates go through ``oracle.ta.resample`` exactly like ``fast_se_metrics/base.py:19-20``).
Differences, all documented in DESIGN.md:

* ``normalize`` (STOI.py:113-119) adds ``1e-12 * randn`` after centring -- a
  nondeterministic term that is below float32 resolution for non-degenerate rows.  The
  oracle takes it in expectation: the noise averages out of the correlations and adds
  N * 1e-24 to the expected squared norm (N = 30 frames, or 15 bands for ESTOI's second
  normalisation), so a row normalises to (v - mean) / sqrt(||v - mean||^2 + N * 1e-24):
  unchanged for any row above ~1e-8 in spread, 0 for a zero-variance row (the reference:
  a random unit vector, contributing ~0 on average), ~0 for rows far below the noise
  (inputs at 1e-15 scale: the reference scores that noise, ~0 +- 1e-2), NaN propagated.
  ESTOI's band normalisation also takes the noise the time normalisation left in each element
  (variance 1e-24 / (||v - mean||^2 + 30e-24), x 14/15 after centring) into its expected norm.
* Per-utterance processing (the reference batches and zero-pads to the batch maximum;
  padded frames/segments are masked out by ``num_segments``, STOI.py:183-189, so the
  per-utterance result is the same).

Pinned by ``tests/test_oracle_golden.py`` against ``tests/golden/*.npz``.
"""
from __future__ import annotations

import math

import numpy as np

from . import ta

FS = 10000
WIN = 256
HOP = 128
N_FFT = 512
NBANDS = 15
MIN_FREQ = 150
N_SEG = 30
BETA = -15.0
DYN_RANGE = 40


def octave_band_matrix() -> np.ndarray:
    """STOI.py:26-47 (float64 build, float32 result)."""
    nfreq = N_FFT // 2 + 1
    freqs = np.linspace(0, FS // 2, nfreq, dtype=np.float64)
    k = np.arange(NBANDS, dtype=np.float64)
    lo = MIN_FREQ * np.power(2.0, (2 * k - 1) / 6)
    hi = MIN_FREQ * np.power(2.0, (2 * k + 1) / 6)
    obm = np.zeros((NBANDS, nfreq), dtype=np.float64)
    for i in range(NBANDS):
        il = int(np.argmin(np.abs(freqs - lo[i])))
        ih = int(np.argmin(np.abs(freqs - hi[i])))
        obm[i, il:ih] = 1
    return obm.astype(np.float32)


def band_edges() -> np.ndarray:
    """[15, 2] first / one-past-last bin of every 1/3-octave band."""
    obm = octave_band_matrix()
    out = np.zeros((NBANDS, 2), dtype=np.int64)
    for i in range(NBANDS):
        nz = np.nonzero(obm[i])[0]
        out[i] = (nz[0], nz[-1] + 1)
    return out


def window() -> np.ndarray:
    """STOI.py:24: torch.hann_window(257)[1:] (periodic) in float32."""
    return ta.hann_periodic(WIN + 1)[1:]


def frame_energies_db(x10: np.ndarray) -> np.ndarray:
    """STOI.py:94-99 for one 10 kHz signal -> [n_frames] float32 dB."""
    w = window().astype(np.float64)
    n = (x10.shape[0] - WIN) // HOP + 1
    if n <= 0:
        return np.zeros(0, dtype=np.float32)
    idx = HOP * np.arange(n)[:, None] + np.arange(WIN)[None, :]
    fr = x10.astype(np.float64)[idx] * w
    return (20.0 * np.log10(np.sqrt((fr ** 2).sum(axis=1)) + 1e-9)).astype(np.float32)


def remove_silent_frames(x: np.ndarray, y: np.ndarray):
    """STOI.py:88-111 + overlap_and_add (:71-86) for one utterance."""
    w = window().astype(np.float64)
    n = (x.shape[0] - WIN) // HOP + 1
    idx = HOP * np.arange(max(n, 0))[:, None] + np.arange(WIN)[None, :]
    xf = x.astype(np.float64)[idx] * w
    yf = y.astype(np.float64)[idx] * w
    e = frame_energies_db(x)
    keep = (e.max() - DYN_RANGE - e) < 0 if n > 0 else np.zeros(0, bool)
    xf, yf = xf[keep], yf[keep]
    nk = int(keep.sum())
    out_len = (nk + 1) * HOP
    xs = np.zeros(out_len)
    ys = np.zeros(out_len)
    for i in range(nk):
        xs[i * HOP:i * HOP + WIN] += xf[i]
        ys[i * HOP:i * HOP + WIN] += yf[i]
    return xs.astype(np.float32), ys.astype(np.float32), nk, keep


def third_octave_bands(sig: np.ndarray) -> np.ndarray:
    """STOI.py:49-69 + :121-125: tob [15, T] float32, T = 1 + (len - 512) // 128."""
    spec = ta.power_spectrogram(sig, N_FFT, HOP, window())[0]       # [T, 257]
    edges = band_edges()
    tob = np.empty((NBANDS, spec.shape[0]), dtype=np.float64)
    for j in range(NBANDS):
        tob[j] = spec[:, edges[j, 0]:edges[j, 1]].sum(axis=1)
    return np.sqrt(tob.astype(np.float32)).astype(np.float32)


def _normalize(v: np.ndarray, axis: int) -> np.ndarray:
    """STOI.py:113-119 in expectation over its 1e-12 * randn term (module docstring)."""
    v = v - v.mean(axis=axis, keepdims=True)
    return v / np.sqrt((v ** 2).sum(axis=axis, keepdims=True) + v.shape[axis] * 1e-24)


def _estoi_normalize(seg: np.ndarray) -> np.ndarray:
    """STOI.py:178-181 (time, then band normalisation) in expectation over both noise terms."""
    c = seg - seg.mean(axis=2, keepdims=True)
    n2 = (c ** 2).sum(axis=2, keepdims=True) + N_SEG * 1e-24
    a = c / np.sqrt(n2)
    a = a - a.mean(axis=1, keepdims=True)
    q = (a ** 2).sum(axis=1, keepdims=True) + (NBANDS - 1) / NBANDS * (1e-24 / n2).sum(axis=1, keepdims=True) \
        + NBANDS * 1e-24
    return a / np.sqrt(q)


def stoi_one(x: np.ndarray, y: np.ndarray, intermediates: dict | None = None):
    """STOI.py:153-198 for one utterance at 10 kHz -> (stoi, estoi) float64.

    Returns (nan, nan) when fewer than 30 STFT frames remain (the reference warns and
    its batched path then fails; num_segments = 0 gives 0/0 in the batched sum).
    """
    xs, ys, nk, keep = remove_silent_frames(x, y)
    nseg = max((xs.shape[0] - N_FFT) // HOP - N_SEG + 2, 0)
    if intermediates is not None:
        intermediates.update(kept=nk, keep_mask=keep, num_segments=nseg)
    if nseg <= 0:
        return math.nan, math.nan
    tx = third_octave_bands(xs).astype(np.float64)
    ty = third_octave_bands(ys).astype(np.float64)
    if intermediates is not None:
        intermediates.update(tob_clean=tx.astype(np.float32), tob_noisy=ty.astype(np.float32))
    idx = np.arange(nseg)[:, None] + np.arange(N_SEG)[None, :]
    xseg = tx[:, idx].transpose(1, 0, 2)                  # [S, 15, 30]
    yseg = ty[:, idx].transpose(1, 0, 2)
    # equalize_clip (STOI.py:129-139)
    alpha = np.sqrt((xseg ** 2).sum(axis=2, keepdims=True)) / (np.sqrt((yseg ** 2).sum(axis=2, keepdims=True)) + 1e-9)
    clip = 10 ** (-BETA / 20)
    yeq = np.minimum(yseg * alpha, xseg * (1 + clip))
    # STOI: normalise over time (dim 3 of the batched tensor)
    cs = _normalize(xseg, 2)
    ds = _normalize(yeq, 2)
    stoi_sum = (cs * ds).sum() / NBANDS
    # ESTOI: time then band normalisation of the un-clipped segments
    ce = _estoi_normalize(xseg)
    de = _estoi_normalize(yseg)
    estoi_sum = (ce * de).sum() / N_SEG
    if intermediates is not None:
        intermediates.update(stoi_seg=(cs * ds).sum(axis=(1, 2)) / NBANDS,
                             estoi_seg=(ce * de).sum(axis=(1, 2)) / N_SEG)
    return stoi_sum / nseg, estoi_sum / nseg


def stoi(clean: np.ndarray, noisy: np.ndarray, sample_rate: int = FS, intermediates: list | None = None):
    """Batched API-equivalent: [B, L] at ``sample_rate`` -> (stoi[B], estoi[B])."""
    clean = np.atleast_2d(np.asarray(clean, dtype=np.float32))
    noisy = np.atleast_2d(np.asarray(noisy, dtype=np.float32))
    if sample_rate != FS:
        clean = ta.resample(clean, sample_rate, FS)
        noisy = ta.resample(noisy, sample_rate, FS)
    s = np.empty(clean.shape[0])
    e = np.empty(clean.shape[0])
    for b in range(clean.shape[0]):
        d = {} if intermediates is not None else None
        s[b], e[b] = stoi_one(clean[b], noisy[b], d)
        if intermediates is not None:
            intermediates.append(d)
    return s, e
