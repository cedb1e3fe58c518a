"""GPU-box: STOI / ESTOI of sinusoid pairs (nearly constant envelope rows, the ill-conditioned case
of DESIGN.md section 9 item 7) from the engine vs the oracle (float64 segment math).

    python tools/probes/tone_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from oracle import stoi_oracle  # noqa: E402
from fast_speech_enhancement_metrics_amd import STOI  # noqa: E402

rng = np.random.default_rng(7)
L = 30000
t = np.arange(L) / 10000.0
c, d = [], []
for f in (250.0, 1000.0, 3150.0):
    tone = np.sin(2 * np.pi * f * t).astype(np.float32)
    c += [tone, tone + 0.05 * rng.standard_normal(L).astype(np.float32)]
    d += [tone + 1e-3 * rng.standard_normal(L).astype(np.float32), tone]
c, d = np.stack(c), np.stack(d)
s64, e64 = stoi_oracle.stoi(c, d, 10000)
s, e = STOI(10000, use_gpu=True).scores(torch.from_numpy(c).cuda(), torch.from_numpy(d).cuda())
s, e = s.cpu().numpy(), e.cpu().numpy()
print("oracle STOI ", np.round(s64, 5), "\nengine STOI ", np.round(s, 5))
print("oracle ESTOI", np.round(e64, 5), "\nengine ESTOI", np.round(e, 5))
print(f"max |dSTOI| {np.max(np.abs(s - s64)):.2e}  max |dESTOI| {np.max(np.abs(e - e64)):.2e}")
