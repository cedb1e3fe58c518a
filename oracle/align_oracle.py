"""ORACLE / TEST INFRASTRUCTURE ONLY -- float64 restatement of the engine's opt-in time alignment
(SURVEY.md 8(f)4).  PARITY UNPINNED against ITU-T P.862 / ludlows' pesq: the reference has no
time alignment (``fast_se_metrics/PESQ.py:19-22``: "1. no time alignment") and no P.862
implementation is importable here, so this module restates the published P.862 section 10
structure as the engine implements it, and the tests pin the engine to it on inputs with a
known delay (``tests/test_align_cpu.py``, ``tests/test_align_gpu.py``):

1. Voice-activity envelopes on 4 ms frames (64 samples at 16 kHz, P.862's ``Downsample``):
   frame energies E[k] = sum of x^2 over the frame; a noise threshold re-estimated 12 times from
   the frames at or below it (mean + 2 standard deviations, times 1.001), starting at mean(E);
   envelope env[k] = log(E[k] / thr) above the threshold, else 0 (P.862 ``apply_VAD``).
2. Crude delay: the lag (in frames, |j| <= M) maximising the plain cross-correlation
   sum_k env_ref[k] env_deg[k + j] (P.862 ``crude_align``); 0 if no lag correlates positively.
3. Fine delay: within +-383 samples of the crude one (P.862 searches +-512 around it at
   16 kHz), the sample lag maximising the cross-correlation of the first differences
   w[n] = x[n] - x[n-1] (n >= 1) of the two signals (a pre-whitened whole-signal form of P.862's
   per-utterance ``time_align`` histogram, which this build does not split into utterances); the
   crude delay if no lag correlates positively.  The window: the crude stage's error on the
   synthetic speech-like pairs reaches ~290 samples (4 ms frames of smooth syllabic envelopes);
   narrower windows, or a decimated intermediate stage, lock onto neighbouring pitch-period peaks
   (measured while choosing the design: +-64 recovered 12 / 24 delays, a decimate-by-4 stage
   248 / 256, the full-rate +-383 window 256 / 256).
4. Delay D > 0 means the degraded signal lags the reference: deg[n] ~ ref[n - D].  The aligned
   degraded row is a[n] = deg[n + D] where 0 <= n + D < L, else 0.

Ties: the first maximum in increasing lag order.
"""
from __future__ import annotations

import numpy as np

FRAME = 64        # samples per envelope frame at 16 kHz (4 ms)
FINE = 383        # fine search half-width in samples (767 lags)
VAD_ITERS = 12


def envelope(x: np.ndarray) -> np.ndarray:
    """VAD log-envelope of one row (step 1)."""
    x = np.asarray(x, dtype=np.float64)
    nfr = x.shape[0] // FRAME
    if nfr == 0:
        return np.zeros(0)
    e = np.square(x[:nfr * FRAME].reshape(nfr, FRAME)).sum(axis=1)
    thr = e.mean()
    for _ in range(VAD_ITERS):
        noise = e[e <= thr]
        if noise.size == 0:
            break
        mu = noise.mean()
        sd = np.sqrt(np.mean(np.square(noise - mu)))
        thr = 1.001 * (mu + 2.0 * sd)
    env = np.zeros(nfr)
    above = e > thr
    env[above] = np.log(e[above] / thr)
    return env


def crude_delay(env_r: np.ndarray, env_d: np.ndarray, max_frames: int) -> int:
    """Step 2: crude delay in frames."""
    nfr = min(env_r.shape[0], env_d.shape[0])
    M = min(max_frames, nfr - 1)
    best, arg = 0.0, 0
    for j in range(-M, M + 1):
        if j >= 0:
            c = float(np.dot(env_r[:nfr - j], env_d[j:nfr]))
        else:
            c = float(np.dot(env_r[-j:nfr], env_d[:nfr + j]))
        if c > best:
            best, arg = c, j
    return arg


def fine_delay(ref: np.ndarray, deg: np.ndarray, d0: int) -> int:
    """Step 3: sample delay within +-FINE of d0 (first differences, n >= 1 on both sides)."""
    r = np.asarray(ref, dtype=np.float64)
    d = np.asarray(deg, dtype=np.float64)
    L = r.shape[0]
    wr = np.zeros(L)
    wd = np.zeros(L)
    wr[1:] = np.diff(r)
    wd[1:] = np.diff(d)
    best, arg = 0.0, d0
    for D in range(d0 - FINE, d0 + FINE + 1):
        lo, hi = max(1, 1 - D), min(L, L - D)
        if hi <= lo:
            continue
        c = float(np.dot(wr[lo:hi], wd[lo + D:hi + D]))
        if c > best:
            best, arg = c, D
    return arg


def delay(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000) -> int:
    """Delay (samples) of one row pair of equal length at 16 kHz."""
    env_r, env_d = envelope(ref), envelope(deg)
    jc = crude_delay(env_r, env_d, -(-max_delay // FRAME))  # 0 for rows under two frames
    return fine_delay(ref, deg, FRAME * jc)


def shift(deg: np.ndarray, D: int) -> np.ndarray:
    """Step 4: the aligned degraded row."""
    L = deg.shape[0]
    out = np.zeros_like(deg)
    lo, hi = max(0, -D), min(L, L - D)
    if hi > lo:
        out[lo:hi] = deg[lo + D:hi + D]
    return out


def align(ref: np.ndarray, deg: np.ndarray, max_delay: int = 16000, lengths=None):
    """(aligned deg [B, L], delays [B]) for [B, L] rows; rows past lengths[b] stay zero."""
    ref = np.atleast_2d(ref)
    deg = np.atleast_2d(deg)
    B, L = ref.shape
    out = np.zeros_like(deg)
    ds = np.zeros(B, dtype=np.int64)
    for b in range(B):
        n = L if lengths is None else int(min(max(lengths[b], 0), L))
        ds[b] = delay(ref[b, :n], deg[b, :n], max_delay)
        out[b, :n] = shift(deg[b, :n], int(ds[b]))
    return out, ds
