"""Cost of the drop-in call's host side at the bench size: PESQ_STOI.scores + one copy vs the
drop-in ``metric(clean, denoised) -> list[dict]`` (benchmark_metrics.py:72-75 times the latter),
and the list-of-dict build alone on host floats (Python dict displays over tolist() vs the
native builder the call uses, csrc/score_list.c).

    python tools/probes/dropin_cost.py [--batch 4096] [--length 160000] [--reps 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ_STOI, _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, a.length, 16000, seed=42, device="cuda")
m = PESQ_STOI(16000, use_gpu=True)


def timeit(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.reps * 1e3


out = {"batch": a.batch, "length": a.length}
out["scores_plus_copy_ms"] = timeit(lambda: torch.stack(m.scores(c, n)).cpu())
for rows in (0, 2048, 1024):
    m.pipeline_rows = rows
    out[f"dropin_call_ms_pipeline_{rows}"] = timeit(lambda: m(c, n))
m.pipeline_rows = 2048
host = torch.stack(m.scores(c, n)).cpu()
t0 = time.perf_counter()
for _ in range(a.reps):
    p, s, e = host.tolist()
    lst = [{"PESQ": x, "STOI": y, "ESTOI": z} for x, y, z in zip(p, s, e)]
out["list_build_python_ms"] = (time.perf_counter() - t0) / a.reps * 1e3
t0 = time.perf_counter()
for _ in range(a.reps):
    lst2 = _native.score_list(host, ("PESQ", "STOI", "ESTOI"))
out["list_build_native_ms"] = (time.perf_counter() - t0) / a.reps * 1e3
assert lst2 == lst
print(json.dumps(out))
