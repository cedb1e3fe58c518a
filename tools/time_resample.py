"""Time the resampler (csrc/resample.hip) of the library named by FSEM_LIB on config-5 shapes:
1024 rows x 30 s at 8 kHz, 8 -> 16 kHz and 8 -> 10 kHz, whole rows and ragged rows (lengths
U[2, 30] s).  Reports ms per call and the algorithmic HBM rate (input read + output written).

    FSEM_LIB=path/to/variant.so python tools/time_resample.py [--reps 20]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd.resample import Resample  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rows", type=int, default=1024)
a = ap.parse_args()
R, L = a.rows, 240000
x = torch.randn(R, L, device="cuda")
lens_np = np.random.default_rng(0).integers(16000, L + 1, size=R).astype(np.int32)
lens = torch.from_numpy(lens_np).cuda()


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / a.reps


for orig, new in ((8000, 16000), (8000, 10000)):
    m = Resample(orig, new).cuda()
    n_out = m.output_length(L)
    for name, ln in (("whole", None), ("ragged", lens)):
        ms = timeit(lambda: m(x, ln))
        rd = 4.0 * (R * L if ln is None else float(lens_np.sum()))
        wr = 4.0 * R * n_out
        print(f"{orig}->{new} {name:6s}: {ms:.3f} ms  {(rd + wr) / ms / 1e9:.2f} TB/s "
              f"(read {rd / 1e9:.2f} GB, write {wr / 1e9:.2f} GB)", flush=True)
