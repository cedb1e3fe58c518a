"""Run one benchmark step (PESQ + STOI on a 10 s @ 16 kHz batch) -- a target for rocprofv3."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--joint", action="store_true", help="one fused PESQ_STOI call instead of two")
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, a.length, device="cuda")
p, s = PESQ(16000, use_gpu=True), STOI(16000, use_gpu=True)
j = PESQ_STOI(16000, use_gpu=True)
# the drop-in call as bench.py times it (one 4096-row engine call, joint.chunk_bounds): per-launch
# counters at the roofline's size (PMC_ROWS in the drivers)
for _ in range(a.reps):
    if a.joint:
        rp = rs = j(c, n)
    else:
        rp, rs = p(c, n), s(c, n)
torch.cuda.synchronize()
print("PESQ[0]", rp[0], "STOI[0]", rs[0])
