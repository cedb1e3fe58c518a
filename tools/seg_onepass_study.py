"""CPU study for DESIGN.md section 9 item 7: would a one-pass (sum / sum-of-squares) form of
stoi_seg's per-(segment, band) statistics keep STOI / ESTOI within the 5e-4 parity bar?

For each input pair the oracle's 1/3-octave envelopes (oracle/stoi_oracle.py intermediates) are
scored three ways: float64 two-pass (the reference's math), float32 two-pass with sequential
30-term sums (the engine's form: centred sums after the mean), and float32 one-pass
(sum x^2 - 30 mu^2 etc., clamped at 0) for the row statistics shared by STOI and ESTOI.
Inputs: speech-like pairs over SNRs, stationary noise, and sinusoids (near-constant envelope rows,
the cancellation worst case).  Prints the max |delta| vs float64 per form and input family.

    python tools/seg_onepass_study.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from oracle import stoi_oracle  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

NSEG, NB = 30, 15
KCLIP = np.float32(1 + 10 ** (15 / 20))


def seqsum(a, axis):
    """Sequential float32 sum along `axis` (the kernel's one-lane-per-segment loop order)."""
    return np.cumsum(a.astype(np.float32), axis=axis, dtype=np.float32).take(-1, axis=axis)


def rsq(v):
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(v > 0, np.float32(1) / np.sqrt(np.maximum(v, np.float32(0)), dtype=np.float32), np.float32(0))


def scores(tx, ty, onepass):
    S = tx.shape[1] - NSEG + 1
    idx = np.arange(S)[:, None] + np.arange(NSEG)[None, :]
    x = tx[:, idx].transpose(1, 0, 2).astype(np.float32)  # [S, 15, 30]
    y = ty[:, idx].transpose(1, 0, 2).astype(np.float32)
    n = np.float32(NSEG)
    sx, sy = seqsum(x, 2), seqsum(y, 2)
    sxx, syy = seqsum(x * x, 2), seqsum(y * y, 2)
    alpha = np.sqrt(sxx) / (np.sqrt(syy) + np.float32(1e-9))
    c = np.minimum(y * alpha[..., None], x * KCLIP)
    mx, my, mc = sx / n, sy / n, seqsum(c, 2) / n
    if onepass:
        dxx = np.maximum(sxx - n * mx * mx, 0)
        dyy = np.maximum(syy - n * my * my, 0)
        dcc = np.maximum(seqsum(c * c, 2) - n * mc * mc, 0)
        dxc = seqsum(x * c, 2) - n * mx * mc
    else:
        d, dy, dc = x - mx[..., None], y - my[..., None], c - mc[..., None]
        dxx, dyy, dcc, dxc = seqsum(d * d, 2), seqsum(dy * dy, 2), seqsum(dc * dc, 2), seqsum(d * dc, 2)
    rx, ry, rc = rsq(dxx), rsq(dyy), rsq(dcc)
    st = (dxc * rx * rc).astype(np.float64).sum() / NB / S
    # ESTOI: rows normalised with (rx, ry), then columns (two-pass, as the engine)
    a = (x - mx[..., None]) * rx[..., None]
    b = (y - my[..., None]) * ry[..., None]
    a = a - a.mean(axis=1, keepdims=True, dtype=np.float32)
    b = b - b.mean(axis=1, keepdims=True, dtype=np.float32)
    ra, rb = rsq(seqsum(a * a, 1)), rsq(seqsum(b * b, 1))
    et = (seqsum(a * b, 1) * ra * rb).astype(np.float64).sum() / NSEG / S
    return st, et


def family(name, pairs):
    worst = {"two-pass f32": [0.0, 0.0], "one-pass f32": [0.0, 0.0]}
    for c, d in pairs:
        inter = []
        s64, e64 = stoi_oracle.stoi(c[None], d[None], 10000, intermediates=inter)
        if not np.isfinite(s64[0]):
            continue
        tx, ty = inter[0]["tob_clean"], inter[0]["tob_noisy"]
        for form, onepass in (("two-pass f32", False), ("one-pass f32", True)):
            s, e = scores(tx, ty, onepass)
            worst[form][0] = max(worst[form][0], abs(s - s64[0]))
            worst[form][1] = max(worst[form][1], abs(e - e64[0]))
    for form, (ds, de) in worst.items():
        print(f"{name:28s} {form}: max |dSTOI| {ds:.2e}  max |dESTOI| {de:.2e}")


def main():
    rng = np.random.default_rng(7)
    L = 30000  # 3 s at 10 kHz
    c, n, _ = speech_like_pairs(8, L, 10000, seed=3)
    family("speech-like, SNR -5..25 dB", list(zip(c.numpy(), n.numpy())))
    noise = [(rng.standard_normal(L).astype(np.float32), rng.standard_normal(L).astype(np.float32)) for _ in range(4)]
    family("stationary white noise", noise)
    t = np.arange(L) / 10000.0
    tones = []
    for f in (250.0, 1000.0, 3150.0):
        tone = np.sin(2 * np.pi * f * t).astype(np.float32)
        tones.append((tone, tone + 1e-3 * rng.standard_normal(L).astype(np.float32)))
        tones.append((tone + 0.05 * rng.standard_normal(L).astype(np.float32), tone))
    family("sinusoids (+ small noise)", tones)


if __name__ == "__main__":
    main()
