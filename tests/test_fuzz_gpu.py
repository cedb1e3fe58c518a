"""Seeded randomized parity sweep of the drop-in API against the oracle.

Each case draws a batch size, an input rate (every common rate the engine resamples), an
utterance length, ragged per-row lengths (some rows too short for PESQ or STOI), an amplitude
scale and a row stride, then scores the batch through ``PESQ``, ``STOI`` and ``PESQ_STOI`` on the
GPU and compares every row with the oracle (the CPU restatement of the reference, pinned by
tests/golden) run on that unpadded row alone -- the definition of a ragged row's result
(batching.py).  Tolerances as tests/test_gpu_parity.py: PESQ 5e-3 (the reference's CPU-vs-GPU
bound, tests/test_cuda.py:23), STOI / ESTOI 5e-4 (its pystoi bound, tests/reference/test_stoi.py);
rows the reference rejects when called alone must be NaN.  The joint entry must give the same
numbers as the two metrics (bitwise).
"""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle, ta

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4
RATES = [8000, 11025, 16000, 22050, 32000, 44100, 48000]


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    sr = int(rng.choice(RATES))
    B = int(rng.integers(1, 9))
    L = int(rng.uniform(1.2, 4.5) * sr)
    ragged = bool(rng.integers(0, 2))
    lens = np.full(B, L, dtype=np.int64)
    if ragged:
        lens = rng.integers(int(0.05 * L), L + 1, size=B)
        lens[rng.integers(0, B)] = L  # one full-capacity row
    scale = float(rng.choice([1e-2, 1.0, 30.0]))
    pad = int(rng.choice([0, 3, 64]))  # extra row stride
    return sr, B, L, lens, ragged, scale, pad


def _oracle_row(c, n, sr):
    """Reference semantics for one unpadded row: PESQ on the row resampled to 16 kHz (NaN where the
    reference's unfold rejects it), STOI/ESTOI at 10 kHz (NaN without a 30-frame segment)."""
    c16 = c if sr == 16000 else ta.resample(c[None], sr, 16000)[0]
    n16 = n if sr == 16000 else ta.resample(n[None], sr, 16000)[0]
    L16 = c16.shape[-1]
    Lp = L16 + L16 % 256
    F = 1 + (Lp - 512) // 256 if Lp >= 512 else 0
    p = float(pesq_oracle.pesq(c16[None], n16[None])[0]) if F >= 20 else float("nan")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            s, e = stoi_oracle.stoi(c[None], n[None], sr)
            s, e = float(s[0]), float(e[0])
        except Exception:  # shorter than one 10 kHz frame
            s, e = float("nan"), float("nan")
    return p, s, e


def _close(got, want, tol, what):
    got, want = np.asarray(got, dtype=np.float64), np.asarray(want, dtype=np.float64)
    np.testing.assert_array_equal(np.isnan(got), np.isnan(want), err_msg=f"{what}: NaN pattern")
    ok = ~np.isnan(want)
    np.testing.assert_allclose(got[ok], want[ok], atol=tol, rtol=0, err_msg=what)


@pytest.mark.parametrize("seed", range(24))
def test_random_batches_vs_oracle(seed):
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    sr, B, L, lens, ragged, scale, pad = _case(seed)
    c, n, _ = speech_like_pairs(B, L, sr, seed=seed, device="cuda")
    c, n = c * scale, n * scale
    if pad:  # rows inside a wider buffer (row stride L + pad)
        cw = torch.zeros(B, L + pad, device="cuda")
        nw = torch.zeros(B, L + pad, device="cuda")
        cw[:, :L], nw[:, :L] = c, n
        c, n = cw[:, :L], nw[:, :L]
    lt = torch.as_tensor(lens, dtype=torch.int32) if ragged else None
    res_p = PESQ(sr, use_gpu=True)(c, n, lengths=lt)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            res_s = STOI(sr, use_gpu=True)(c, n, lengths=lt)
        except TypeError:  # no row has a STOI segment: the reference's failure mode (STOI.py:162-165)
            res_s = [{"STOI": float("nan"), "ESTOI": float("nan")}] * B
        res_j = PESQ_STOI(sr, use_gpu=True)(c, n, lengths=lt)
    gp = [d["PESQ"] for d in res_p]
    gs = [d["STOI"] for d in res_s]
    ge = [d["ESTOI"] for d in res_s]
    cc, nn = c.cpu().numpy(), n.cpu().numpy()
    want = np.array([_oracle_row(cc[b, :lens[b]], nn[b, :lens[b]], sr) for b in range(B)])
    tag = f"seed {seed}: sr {sr} B {B} L {L} ragged {ragged} scale {scale} pad {pad}"
    _close(gp, want[:, 0], PESQ_TOL, f"PESQ {tag}")
    _close(gs, want[:, 1], STOI_TOL, f"STOI {tag}")
    _close(ge, want[:, 2], STOI_TOL, f"ESTOI {tag}")
    for key, ref in (("PESQ", gp), ("STOI", gs), ("ESTOI", ge)):
        np.testing.assert_array_equal(np.array([d[key] for d in res_j]), np.array(ref), err_msg=f"joint {key} {tag}")
