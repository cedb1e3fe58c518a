"""Interleaved A/B of the drop-in call PESQ_STOI(16000, use_gpu=True)(clean, noisy) -> list of
dicts, timed as bench.py times it (wall clock over back-to-back calls, the result dropped each
time): the fast path (joint.py _fast_call) against the generic path, and the fast path with its
scores copied from a device buffer (host_scores = False) against written straight into mapped
pinned memory, in one process.

    python tools/probes/ab_dropin_fast.py [--batch 4096] [--steps 20] [--rounds 6]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ_STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, a.length, 16000, seed=42, device="cuda")
fast = PESQ_STOI(16000, use_gpu=True)
slow = PESQ_STOI(16000, use_gpu=True)
slow._fast_ok = lambda *x: False
copy = PESQ_STOI(16000, use_gpu=True)
copy.host_scores = False
for m in (fast, slow, copy):
    for _ in range(5):
        m(c, n)
torch.cuda.synchronize()
t = {"fast": [], "generic": [], "fast_copy": []}
order = [("fast", fast), ("generic", slow), ("fast_copy", copy)]
for r in range(a.rounds):
    for name, m in (order if r % 2 == 0 else order[::-1]):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m(c, n)
        torch.cuda.synchronize()
        t[name].append((time.perf_counter() - t0) / a.steps * 1e3)
for name, v in t.items():
    print(f"{name}: median {statistics.median(v):.4f} ms per call  min {min(v):.4f}  max {max(v):.4f}  "
          f"({a.batch / statistics.median(v) * 1e3:,.0f} utt/s)")
print("equal lists:", fast(c, n) == slow(c, n) == copy(c, n))
