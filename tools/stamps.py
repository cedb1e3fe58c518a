"""Phase shares of pesq_front from the s_memtime stamps of the diagnostic build.

    FSEM_LIB=fast_speech_enhancement_metrics_amd/lib/libfsem_stamps.so python tools/stamps.py
Never quote this build's run time: read its shares only.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

assert "stamps" in _native.LIB_PATH, "run with FSEM_LIB=.../libfsem_stamps.so"
B = int(os.environ.get("B", "4096"))
c, n, _ = speech_like_pairs(B, 160000, device="cuda")
m = (PESQ_STOI if os.environ.get("JOINT") else PESQ)(16000, use_gpu=True)  # JOINT=1: pesq_front<true>
m(c, n)
m(c, n)
lib = _native.load()
buf = np.zeros((65536, 16), dtype=np.uint64)
fn = lib.fsem_debug_read_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
assert fn(buf.ctypes.data, buf.nbytes) == 0
st = buf.astype(np.float64)
segs = [("tile->LDS", 0, 14), ("resample", 14, 1), ("IIR pass1", 1, 2), ("scan", 2, 3), ("IIR pass2", 3, 4),
        ("fft r0", 4, 6)] + [(f"fft r{r}", 5 + r, 6 + r) for r in range(1, 7)] + [("mfma bark", 13, 15)]
valid = (st[:, 15] > 0) & (st[:, 0] > 0)
tot = (st[valid, 15] - st[valid, 0]).mean()
print(f"blocks {valid.sum()}, mean item time {tot:.0f} cycles (s_memtime ticks)")
for nm, a, b in segs:
    ok = valid & (st[:, a] > 0) & (st[:, b] > 0)
    d = (st[ok, b] - st[ok, a]).mean() if ok.any() else 0
    print(f"  {nm:16s} {d:10.0f}  {100 * d / tot:5.1f}%")
