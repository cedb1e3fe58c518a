"""Per-call latency and utterances/s of the drop-in API at the reference's own benchmark setting
(benchmark_metrics.py:17-20: 16 s clips at 16 kHz, batch 64): metric(clean, denoised)
-> list of dicts, inputs already on the device, first calls dropped.

    python tools/probes/small_batch.py [--batch 64] [--seconds 16] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--seconds", type=float, default=16.0)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, int(a.seconds * 16000), 16000, device="cuda")
out = {"batch": a.batch, "seconds": a.seconds}
for name, m in (("PESQ", PESQ(16000, use_gpu=True)), ("STOI", STOI(16000, use_gpu=True)),
                ("PESQ_STOI", PESQ_STOI(16000, use_gpu=True))):
    for _ in range(3):
        m(c, n)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        r = m(c, n)
    dt = (time.perf_counter() - t0) / a.reps
    out[name] = {"ms_per_call": round(dt * 1e3, 3), "utterances_per_s": round(a.batch / dt, 1)}
print(json.dumps(out))
