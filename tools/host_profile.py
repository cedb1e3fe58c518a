"""Host-side cost of one drop-in call at small batch (cProfile over repeated calls), and the
launch-only time of scores() (no host sync), to size the per-call host overhead.

    python tools/host_profile.py [--batch 64] [--seconds 16] [--metric PESQ_STOI]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import fast_speech_enhancement_metrics_amd as fsem  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--seconds", type=float, default=16.0)
ap.add_argument("--metric", default="PESQ_STOI")
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, int(a.seconds * 16000), 16000, device="cuda")
m = getattr(fsem, a.metric)(16000, use_gpu=True)
for _ in range(5):
    m(c, n)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    m.scores(c, n) if a.metric != "STOI" else m.scores(c, n, 16000)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"scores() launch-only {1e3 * (t1 - t0) / a.reps:.3f} ms/call; queue drained after {1e3 * (t2 - t0) / a.reps:.3f} ms/call")
t0 = time.perf_counter()
for _ in range(a.reps):
    m(c, n)
print(f"__call__ {1e3 * (time.perf_counter() - t0) / a.reps:.3f} ms/call")
pr = cProfile.Profile()
pr.enable()
for _ in range(a.reps):
    m(c, n)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
