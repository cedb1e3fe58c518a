"""The drop-in call's row chunking at the bench size: the list of dicts of chunk k is built
while chunk k+1's kernels run, so only the last chunk's list is exposed, at the price of one
more engine call per chunk.  Times PESQ_STOI(16000, use_gpu=True)(clean, noisy) with several
chunk plans (interleaved rounds, medians) and checks every plan returns the same list.

    python tools/probes/ab_dropin_chunks.py [--rounds 8] [--reps 5]
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
ap.add_argument("--rounds", type=int, default=8)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
B, L = 4096, 160000
c, n, _ = speech_like_pairs(B, L, 16000, seed=42, device="cuda")
m = PESQ_STOI(16000, use_gpu=True)
plans = {
    "1x4096": [(0, 4096)],
    "2x2048": [(0, 2048), (2048, 4096)],
    "2560+1536": [(0, 2560), (2560, 4096)],
    "2048+1536+512": [(0, 2048), (2048, 3584), (3584, 4096)],
    "3072+1024": [(0, 3072), (3072, 4096)],
}
orig = m.chunk_bounds


def call(plan):
    m.chunk_bounds = lambda batch, on_gpu=True: plans[plan]
    try:
        return m(c, n)
    finally:
        m.chunk_bounds = orig


ref = call("2x2048")
for p in plans:
    got = call(p)
    # chunks of <= 2 rows per CU use the 4-wave PESQ back end (summation order only, <= 1e-5)
    dev = max(abs(g[k] - r[k]) for g, r in zip(got, ref) for k in r)
    assert dev <= 2e-5, (p, dev)
    print(f"{p}: max |d| vs 2x2048 {dev:.2e}")
times = {p: [] for p in plans}
for r in range(a.rounds):
    order = list(plans)[r % len(plans):] + list(plans)[:r % len(plans)]
    for p in order:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            call(p)
        torch.cuda.synchronize()
        times[p].append((time.perf_counter() - t0) / a.reps * 1e3)
for p in plans:
    med = statistics.median(times[p])
    print(f"{p:>15}: median {med:.3f} ms per call ({B / med * 1e3:,.0f} utt/s)  min {min(times[p]):.3f}")
