"""Edge cases of the HIP engine against the oracle (the CPU restatement pinned to the
reference's golden vectors): the shortest inputs each metric accepts, the PESQ.py:128
padding quirk around multiples of 256, segment-boundary lengths of the PESQ front end's
tiling, a single utterance, all-silent / identical signals, and a ragged batch whose rows
sit on those boundaries.  Sizes are small so the oracle finishes in seconds."""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4


def _pairs(B, L, seed, sr=16000):
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(B, L, sr, seed=seed, snr_low=0, snr_high=30)
    return c, n


def _stoi_oracle(c, n, sr=16000):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return stoi_oracle.stoi(c.numpy(), n.numpy(), sr)


# 5248 + 5248 % 256 = 5376 -> exactly 20 frames; 5376 -> 20; 5375 (pad 255) -> 21;
# 12544 / 12545: one PESQ front-end tile exactly / one sample into the second segment
@pytest.mark.parametrize("L", [5248, 5376, 5375, 12544, 12545, 25089])
def test_pesq_boundary_lengths_vs_oracle(L):
    from fast_speech_enhancement_metrics_amd import PESQ
    c, n = _pairs(2, L, seed=L)
    got = np.array([r["PESQ"] for r in PESQ(16000, use_gpu=True)(c, n)])
    np.testing.assert_allclose(got, pesq_oracle.pesq(c.numpy(), n.numpy()), atol=PESQ_TOL, rtol=0)


def test_pesq_too_short_raises_like_reference():
    from fast_speech_enhancement_metrics_amd import PESQ
    c, n = _pairs(1, 5247, seed=3)  # 5247 + 127 = 5374 -> 19 frames
    with pytest.raises(RuntimeError):
        PESQ(16000, use_gpu=True)(c, n)


@pytest.mark.parametrize("L", [16000, 16001, 16003])
def test_stoi_short_and_odd_lengths_vs_oracle(L):
    from fast_speech_enhancement_metrics_amd import STOI
    c, n = _pairs(2, L, seed=L + 1)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        res = STOI(16000, use_gpu=True)(c, n)
    s_o, e_o = _stoi_oracle(c, n)
    got_s = np.array([r["STOI"] for r in res])
    got_e = np.array([r["ESTOI"] for r in res])
    assert np.array_equal(np.isnan(got_s), np.isnan(s_o))
    m = ~np.isnan(s_o)
    np.testing.assert_allclose(got_s[m], s_o[m], atol=STOI_TOL, rtol=0)
    np.testing.assert_allclose(got_e[m], e_o[m], atol=STOI_TOL, rtol=0)


def test_single_utterance_1d_input():
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    c, n = _pairs(1, 48000, seed=9)
    p = PESQ(16000, use_gpu=True)(c[0], n[0])
    s = STOI(16000, use_gpu=True)(c[0], n[0])
    assert len(p) == 1 and len(s) == 1
    assert abs(p[0]["PESQ"] - pesq_oracle.pesq(c.numpy(), n.numpy())[0]) < PESQ_TOL
    assert abs(s[0]["STOI"] - _stoi_oracle(c, n)[0][0]) < STOI_TOL


def test_identical_signals_score_high():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, _ = _pairs(2, 48000, seed=11)
    res = PESQ_STOI(16000, use_gpu=True)(c, c.clone())
    op = pesq_oracle.pesq(c.numpy(), c.numpy())
    for r, o in zip(res, op):
        assert abs(r["PESQ"] - o) < PESQ_TOL and r["PESQ"] > 4.4
        assert r["STOI"] > 0.999 and r["ESTOI"] > 0.999


def test_ragged_rows_on_boundaries_vs_oracle():
    """One ragged batch whose rows sit on the boundaries above, each row vs the oracle alone."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    lens = [5248, 5375, 12544, 12545, 25089, 48000, 16001]
    cap = max(lens)
    c, n = _pairs(len(lens), cap, seed=21)
    rows_c = [c[i, :L] for i, L in enumerate(lens)]
    rows_n = [n[i, :L] for i, L in enumerate(lens)]
    res = PESQ_STOI(16000, use_gpu=True)(rows_c, rows_n)
    for i, L in enumerate(lens):
        op = pesq_oracle.pesq(rows_c[i][None].numpy(), rows_n[i][None].numpy())[0]
        so, eo = _stoi_oracle(rows_c[i][None], rows_n[i][None])
        assert abs(res[i]["PESQ"] - op) < PESQ_TOL, (L, res[i], op)
        if np.isnan(so[0]):
            assert np.isnan(res[i]["STOI"])
        else:
            assert abs(res[i]["STOI"] - so[0]) < STOI_TOL and abs(res[i]["ESTOI"] - eo[0]) < STOI_TOL, (L, res[i])
