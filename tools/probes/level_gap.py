"""STOI / ESTOI / PESQ when the denoised signal sits far below the clean one (relative scale
1e-3 .. 1e-9), and the reverse, against the oracle: probes the shared complex FFT's cross-talk
(clean + i*denoised in one FFT) at large level gaps.

    python tools/probes/level_gap.py
"""
import os
import sys
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ, STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402
from oracle import pesq_oracle, stoi_oracle  # noqa: E402

c, n, _ = speech_like_pairs(4, 48000, 16000, seed=9, device="cuda")
st = STOI(16000, use_gpu=True)
pq = PESQ(16000, use_gpu=True)
warnings.simplefilter("ignore")
for a, b in [(1.0, 1e-3), (1.0, 1e-5), (1.0, 1e-7), (1.0, 1e-9), (1e-7, 1.0)]:
    cc, nn = c * a, n * b
    s, e = st.scores(cc, nn, 16000)
    p = pq.scores(cc, nn)
    os_, oe = stoi_oracle.stoi(cc.cpu().numpy(), nn.cpu().numpy(), 16000)
    op = pesq_oracle.pesq(cc.cpu().numpy(), nn.cpu().numpy())
    print(f"clean x{a:g} denoised x{b:g}: |dSTOI| {np.abs(s.cpu().numpy() - os_).max():.2e} "
          f"|dESTOI| {np.abs(e.cpu().numpy() - oe).max():.2e} |dPESQ| {np.abs(p.cpu().numpy() - op).max():.2e}  "
          f"STOI {np.round(os_, 4)}")
