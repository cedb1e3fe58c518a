"""Clean and denoised signals at very different levels.  The STOI engine transforms clean and
denoised frames together in one complex FFT (stoi_tob), whose rounding leaks ~1e-7 of the louder
spectrum into the quieter one; frames with a large peak gap are equalised by an exact power of
two first.  Here the denoised rows sit 60-180 dB below the clean ones (e.g. int16-scaled clean
against float denoised), the reverse, and a denoised row quiet only over a stretch of ~80 frames,
all against the oracle (the CPU restatement of the reference, pinned by tests/golden) within the
parity tolerances of tests/test_gpu_parity.py, through STOI and the joint entry."""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4


@pytest.fixture(scope="module")
def pairs():
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    return speech_like_pairs(4, 48000, 16000, seed=9, device="cuda")[:2]


@pytest.mark.parametrize("a,b", [(1.0, 1e-3), (1.0, 1e-5), (1.0, 1e-7), (1.0, 1e-9), (1e-7, 1.0),
                                 (32768.0, 1.0), (1.0, 32768.0)])
def test_global_level_gap(pairs, a, b):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI, STOI
    c, n = pairs
    cc, nn = c * a, n * b
    s, e = STOI(16000, use_gpu=True).scores(cc, nn, 16000)
    mos, sj, ej = PESQ_STOI(16000, use_gpu=True).scores(cc, nn)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        os_, oe = stoi_oracle.stoi(cc.cpu().numpy(), nn.cpu().numpy(), 16000)
    op = pesq_oracle.pesq(cc.cpu().numpy(), nn.cpu().numpy())
    np.testing.assert_allclose(s.cpu().numpy(), os_, rtol=0, atol=STOI_TOL)
    np.testing.assert_allclose(e.cpu().numpy(), oe, rtol=0, atol=STOI_TOL)
    np.testing.assert_array_equal(sj.cpu().numpy(), s.cpu().numpy())
    np.testing.assert_array_equal(ej.cpu().numpy(), e.cpu().numpy())
    np.testing.assert_allclose(mos.cpu().numpy(), op, rtol=0, atol=PESQ_TOL)


def test_local_level_gap(pairs):
    """Denoised rows 120 dB down over 0.8-1.8 s only (segments inside the stretch see the gap)."""
    from fast_speech_enhancement_metrics_amd import STOI
    c, n = pairs
    nn = n.clone()
    nn[:, 12800:28800] *= 1e-6
    s, e = STOI(16000, use_gpu=True).scores(c, nn, 16000)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        os_, oe = stoi_oracle.stoi(c.cpu().numpy(), nn.cpu().numpy(), 16000)
    np.testing.assert_allclose(s.cpu().numpy(), os_, rtol=0, atol=STOI_TOL)
    np.testing.assert_allclose(e.cpu().numpy(), oe, rtol=0, atol=STOI_TOL)
