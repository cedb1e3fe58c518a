"""STOI / ESTOI of sinusoid pairs against the reference's own outputs (golden `tones_10k`, made by
tests/golden/make_golden.py).  Nearly constant 1/3-octave envelope rows make the per-segment
normalisations ill-conditioned: the reference's float32 rounding alone puts the float64 oracle
3.6e-4 / 7.4e-4 away from it (tests/test_oracle_golden.py), so the speech bar of 5e-4 cannot
apply here.  The engine (float32, hardware rsq, shared complex FFT) measured 7.2e-4 (STOI) and
1.2e-3 (ESTOI) from the reference; the bar below is 2.5e-3, a quarter of BASELINE.json's 0.01."""
import numpy as np
import pytest
import torch

from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
TONE_TOL = 2.5e-3


def test_tones_vs_reference():
    from fast_speech_enhancement_metrics_amd import STOI
    g = load_golden("tones_10k")
    c = torch.from_numpy(g["clean_f"]).cuda()
    n = torch.from_numpy(g["noisy_f"]).cuda()
    res = STOI(int(g["sample_rate"]), use_gpu=True)(c, n)
    np.testing.assert_allclose([r["STOI"] for r in res], g["stoi"], atol=TONE_TOL, rtol=0)
    np.testing.assert_allclose([r["ESTOI"] for r in res], g["estoi"], atol=TONE_TOL, rtol=0)
