"""Non-finite samples.  The reference is plain torch arithmetic, so a NaN / Inf sample poisons
whatever it reaches: in the clean signal it makes the STOI VAD's max energy NaN (no frame kept:
STOI / ESTOI NaN, STOI.py:94-104) and PESQ's level alignment NaN; in the denoised signal it
reaches PESQ always, and STOI only through frames the clean VAD keeps (a NaN band envelope then
runs through equalize_clip / normalize / the correlation sum, STOI.py:113-151).  Other rows of
the batch are untouched.  The oracle agrees except where its normalisation maps a NaN row to 0
(its documented zero-variance rule, oracle/stoi_oracle.py), so that case is checked by the
reference's propagation semantics instead."""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def base():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(3, 48000, 16000, seed=5, device="cuda")
    m = PESQ_STOI(16000, use_gpu=True)
    return c, n, m, [t.cpu().numpy() for t in m.scores(c, n)]


def _run(m, c, n):
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    out = [t.cpu().numpy() for t in m.scores(c, n)]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        p = PESQ(16000, use_gpu=True).scores(c, n).cpu().numpy()
        s, e = (t.cpu().numpy() for t in STOI(16000, use_gpu=True).scores(c, n, 16000))
    for a, b in zip(out, (p, s, e)):  # joint entry == the two metrics, NaN included
        assert np.array_equal(a, b, equal_nan=True)
    return out


def test_nan_in_clean(base):
    c, n, m, ref = base
    cc = c.clone()
    cc[0, 5] = float("nan")
    mos, s, e = _run(m, cc, n)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        os_, oe = stoi_oracle.stoi(cc.cpu().numpy(), n.cpu().numpy(), 16000)
    op = pesq_oracle.pesq(cc.cpu().numpy(), n.cpu().numpy())
    assert np.isnan(mos[0]) and np.isnan(s[0]) and np.isnan(e[0])
    assert np.isnan(op[0]) and np.isnan(os_[0]) and np.isnan(oe[0])
    for k, v in enumerate((mos, s, e)):
        np.testing.assert_array_equal(v[1:], ref[k][1:])


def test_nan_in_denoised_kept_frame(base):
    c, n, m, ref = base
    nn = n.clone()
    nn[1, 24000] = float("nan")  # mid-row: inside frames the clean VAD keeps
    mos, s, e = _run(m, c, nn)
    assert np.isnan(mos[1]) and np.isnan(s[1]) and np.isnan(e[1])
    assert np.isnan(pesq_oracle.pesq(c.cpu().numpy(), nn.cpu().numpy())[1])
    for k, v in enumerate((mos, s, e)):
        np.testing.assert_array_equal(v[[0, 2]], ref[k][[0, 2]])


def test_inf_in_denoised_dropped_frame(base):
    """An Inf inside the silent lead-in the clean VAD drops: STOI unaffected (as the oracle),
    PESQ NaN (as the oracle: the level alignment's power is Inf)."""
    c, n, m, ref = base
    nn = n.clone()
    nn[2, 2000] = float("inf")
    mos, s, e = _run(m, c, nn)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        os_, oe = stoi_oracle.stoi(c.cpu().numpy(), nn.cpu().numpy(), 16000)
    assert np.isnan(mos[2]) and np.isnan(pesq_oracle.pesq(c.cpu().numpy(), nn.cpu().numpy())[2])
    np.testing.assert_allclose(s[2], os_[2], atol=5e-4)
    np.testing.assert_allclose(e[2], oe[2], atol=5e-4)
