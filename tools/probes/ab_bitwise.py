"""Scores of the library named by FSEM_LIB on a fixed synthetic batch, saved for a bitwise A/B.

    FSEM_LIB=.../var/va.so python tools/probes/ab_bitwise.py gpurun_out/a.npy
    FSEM_LIB=.../var/vb.so python tools/probes/ab_bitwise.py gpurun_out/b.npy --compare gpurun_out/a.npy
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ_STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--compare")
ap.add_argument("--batch", type=int, default=1024)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, 160000, device="cuda")
m = PESQ_STOI(16000, use_gpu=True)
s = np.stack([t.cpu().numpy() for t in m.scores(c, n)])
np.save(a.out, s)
if a.compare:
    r = np.load(a.compare)
    same = np.array_equal(s.view(np.uint32), r.view(np.uint32))
    print("bitwise equal" if same else f"DIFFER: max |d| {np.nanmax(np.abs(s - r), axis=1)}")
    sys.exit(0 if same else 1)
