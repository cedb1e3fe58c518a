"""Interleaved A/B of fsem_time_align_f32 (opt-in time alignment) across library variants in one
process on the GPU box, as tools/ab_joint.py: rows with known synthetic delays, each variant
called `--reps` times per round in rotating order, HIP-event timed; checks that every variant
returns the same delays and that they equal the synthetic ones.

    python tools/ab_align.py VAR... [--batch 4096] [--length 160000]
"""
import argparse
import ctypes
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
_vp, _i64, _i32, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
libs = {}
for v in a.variants:
    path = os.path.join(os.path.dirname(__file__), "..", "fast_speech_enhancement_metrics_amd", "lib", "var", v + ".so")
    if v == "head":
        path = _native.LIB_PATH
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    lib.fsem_time_align_workspace_bytes.restype = _sz
    lib.fsem_time_align_workspace_bytes.argtypes = [_i64, _i64]
    lib.fsem_time_align_f32.argtypes = [_vp, _vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _i64, _vp, _sz, _vp]
    libs[v] = lib
B, L = a.batch, a.length
c, n, _ = speech_like_pairs(B, L, 16000, seed=5, device="cuda")
rng = np.random.default_rng(5)
D = torch.from_numpy(rng.integers(-2000, 2001, B)).cuda()
t = torch.arange(L, device="cuda")
src = t[None, :] - D[:, None]
deg = torch.where((src >= 0) & (src < L), n.gather(1, src.clamp(0, L - 1)), torch.zeros_like(n))
del n, src
out = torch.empty(B, L, device="cuda")
ws = _native.workspace(max(lib.fsem_time_align_workspace_bytes(B, L) for lib in libs.values()), c.device)
delays = {v: torch.empty(B, dtype=torch.int32, device="cuda") for v in libs}
h = torch.cuda.current_stream().cuda_stream


def launch(v):
    rc = libs[v].fsem_time_align_f32(c.data_ptr(), deg.data_ptr(), B, L, L, None, 16000, delays[v].data_ptr(),
                                     out.data_ptr(), L, ws.data_ptr(), ws.numel(), h)
    assert rc == 0, rc


for v in libs:
    launch(v)
torch.cuda.synchronize()
times = {v: [] for v in libs}
order = list(libs)
for r in range(a.rounds):
    for v in order[r % len(order):] + order[:r % len(order)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            launch(v)
        e1.record()
        e1.synchronize()
        times[v].append(e0.elapsed_time(e1) / a.reps)
for v in libs:
    ok = int((delays[v].long() == D).sum())
    same = bool(torch.equal(delays[v], delays[order[0]]))
    print(f"{v}: median {statistics.median(times[v]):.3f} ms per {B} x {L} (min {min(times[v]):.3f}); "
          f"delays recovered {ok}/{B}; equal to {order[0]}: {same}")
