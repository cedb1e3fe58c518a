"""Batch sizes past the HIP grid.y limit (65535 rows) and rate pairs whose resampling filter does
not fit the small constant table (44.1 / 22.05 / 11.025 kHz), through the drop-in API.

* Batches: 64 distinct pairs tiled to 65 536 + 3 rows; every row must score bitwise as its source
  row does in a batch of 64 (kernels that map rows to grid.y run in slices of 65 535 rows).  Each
  engine path that used grid.y is covered: the joint entry (stoi_tob), STOI at 16 kHz, 10 kHz
  (stoi_resample_vad) and 8 kHz (tiled resampler + stoi_vad10), PESQ at 8 kHz (8 -> 16 kHz
  resampler).
* Rates: fsem_resample_f32 for the large-table pairs against the oracle's torchaudio restatement
  (oracle/ta.py), and PESQ / STOI / PESQ_STOI at 44.1 kHz against the oracle end to end.  The
  reference has no test at these rates (its tests run at 16 and 10 kHz): the oracle is the only pin.
"""
import ctypes
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle, ta

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4  # engine vs reference (test_gpu_parity.py)
NB = 65536 + 3


def _tiled(sr, seconds, nsrc=64):
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(nsrc, int(seconds * sr), sr, seed=7 + sr, device="cuda")
    reps = -(-NB // nsrc)
    return c, n, c.repeat(reps, 1)[:NB].contiguous(), n.repeat(reps, 1)[:NB].contiguous()


def _assert_tiled_equal(big, small):
    big, small = big.cpu().numpy(), small.cpu().numpy()
    src = np.arange(NB) % small.shape[0]
    np.testing.assert_array_equal(big, small[src])


def test_joint_and_stoi_16k_past_grid_limit():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI, STOI
    c, n, cb, nb = _tiled(16000, 1.0)
    m = PESQ_STOI(16000, use_gpu=True)
    for got, want in zip(m.scores(cb, nb), m.scores(c, n)):
        _assert_tiled_equal(got, want)
    s = STOI(16000, use_gpu=True)
    for got, want in zip(s.scores(cb, nb, 16000), s.scores(c, n, 16000)):
        _assert_tiled_equal(got, want)


@pytest.mark.parametrize("sr", [10000, 8000])
def test_stoi_other_rates_past_grid_limit(sr):
    from fast_speech_enhancement_metrics_amd import STOI
    c, n, cb, nb = _tiled(sr, 1.0)
    s = STOI(sr, use_gpu=True)
    for got, want in zip(s.scores(cb, nb, sr), s.scores(c, n, sr)):
        _assert_tiled_equal(got, want)


def test_pesq_8k_past_grid_limit():
    from fast_speech_enhancement_metrics_amd import PESQ
    c, n, cb, nb = _tiled(8000, 1.0)
    p = PESQ(8000, use_gpu=True)
    _assert_tiled_equal(p.scores(cb, nb, sample_rate=8000), p.scores(c, n, sample_rate=8000))
    out = p(cb[:3], nb[:3])  # the drop-in call agrees with scores()
    want = p.scores(c[:3], n[:3], sample_rate=8000).cpu().numpy()
    np.testing.assert_array_equal(np.array([d["PESQ"] for d in out], dtype=np.float32), want)


BIG_RATES = [(44100, 16000), (22050, 16000), (11025, 16000), (44100, 10000), (22050, 10000), (32000, 10000)]


@pytest.mark.parametrize("orig,new", BIG_RATES)
@pytest.mark.parametrize("n", [1, 37, 4001, 30000])
def test_resample_large_tables_vs_oracle(orig, new, n):
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    rng = np.random.default_rng(n + orig + 3 * new)
    x = rng.standard_normal((3, n)).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    n_out = lib.fsem_resample_length(n, orig, new)
    assert n_out == -(-n * new // orig)
    out = torch.full((3, n_out), float("nan"), device="cuda")
    _native.check(lib.fsem_resample_f32(ctypes.c_void_p(xt.data_ptr()), 3, n, n, ctypes.c_void_p(out.data_ptr()),
                                        n_out, orig, new, ctypes.c_void_p(_native.stream_handle())), "resample")
    got = out.cpu().numpy()
    ref = ta.resample(x, orig, new)
    np.testing.assert_allclose(got, ref, atol=2e-6 * max(1.0, np.abs(ref).max()), rtol=0)


def test_resample_rows_large_table():
    """Ragged rows through the large-table form: each row as the row alone, zero tail."""
    from fast_speech_enhancement_metrics_amd.resample import Resample
    rng = np.random.default_rng(1)
    lens = np.array([20000, 1, 441, 12345, 0, 19999], dtype=np.int32)
    x = rng.standard_normal((len(lens), 20000)).astype(np.float32)
    out = Resample(44100, 16000).cuda()(torch.from_numpy(x).cuda(), torch.from_numpy(lens).cuda()).cpu().numpy()
    for r, ln in enumerate(lens):
        k = -(-int(ln) * 160 // 441)
        if ln:
            ref = ta.resample(x[r:r + 1, :ln], 44100, 16000)[0]
            np.testing.assert_allclose(out[r, :k], ref, atol=2e-6 * max(1.0, np.abs(ref).max()), rtol=0)
        assert (out[r, k:] == 0).all(), r


def test_unsupported_rate_is_rejected():
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    assert lib.fsem_resample_length(1000, 44100, 16001) == -1  # a 44 134-tap filter: FSEM_ERATE
    x = torch.zeros(1, 1000, device="cuda")
    out = torch.zeros(1, 1000, device="cuda")
    rc = lib.fsem_resample_f32(x.data_ptr(), 1, 1000, 1000, out.data_ptr(), 1000, 44100, 16001,
                               _native.stream_handle())
    assert rc == _native.FSEM_ERATE


@pytest.mark.parametrize("sr", [44100, 22050])
def test_metrics_at_cd_rates_vs_oracle(sr):
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(3, int(2.5 * sr), sr, seed=11, device="cuda")
    p = np.array([d["PESQ"] for d in PESQ(sr, use_gpu=True)(c, n)])
    st = STOI(sr, use_gpu=True)(c, n)
    s, e = np.array([d["STOI"] for d in st]), np.array([d["ESTOI"] for d in st])
    j = PESQ_STOI(sr, use_gpu=True)(c, n)
    cc, nn = c.cpu().numpy(), n.cpu().numpy()
    op = pesq_oracle.pesq(ta.resample(cc, sr, 16000), ta.resample(nn, sr, 16000))
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        os_, oe = stoi_oracle.stoi(cc, nn, sr)
    np.testing.assert_allclose(p, op, atol=PESQ_TOL, rtol=0)
    np.testing.assert_allclose(s, os_, atol=STOI_TOL, rtol=0)
    np.testing.assert_allclose(e, oe, atol=STOI_TOL, rtol=0)
    np.testing.assert_array_equal(np.array([d["PESQ"] for d in j]), p)
    np.testing.assert_array_equal(np.array([d["STOI"] for d in j]), s)
