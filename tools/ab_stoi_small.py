"""Interleaved A/B of fsem_stoi_f32 (16 kHz rows, fused 16 -> 10 kHz) at the reference's benchmark
batch (64 x 16 s) across library variants in one process: the engine's per-call latency.

    python tools/ab_stoi_small.py VAR... [--batch 64] [--seconds 16]
"""
import argparse
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--seconds", type=float, default=16.0)
ap.add_argument("--reps", type=int, default=50)
ap.add_argument("--rounds", type=int, default=6)
a = ap.parse_args()
_vp, _i64, _i32, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_size_t
libs = {}
for v in a.variants:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "fast_speech_enhancement_metrics_amd", "lib", "var",
                                   v + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.fsem_stoi_workspace_bytes.restype = _sz
    lib.fsem_stoi_workspace_bytes.argtypes = [_i64, _i64, _i32]
    lib.fsem_stoi_f32.argtypes = [_vp, _vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp, _vp, _sz, _vp]
    libs[v] = lib
B, L = a.batch, int(a.seconds * 16000)
c, n, _ = speech_like_pairs(B, L, 16000, seed=3, device="cuda")
ws = _native.workspace(max(lib.fsem_stoi_workspace_bytes(B, L, 16000) for lib in libs.values()), c.device)
s, e = torch.empty(B, device="cuda"), torch.empty(B, device="cuda")
h = torch.cuda.current_stream().cuda_stream


def call(v):
    assert libs[v].fsem_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, 16000, s.data_ptr(), e.data_ptr(),
                                 ws.data_ptr(), ws.numel(), h) == 0


times = {v: [] for v in libs}
order = list(libs)
for v in order:
    for _ in range(5):
        call(v)
torch.cuda.synchronize()
for r in range(a.rounds):
    for v in order[r % len(order):] + order[:r % len(order)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            call(v)
        e1.record()
        e1.synchronize()
        times[v].append(e0.elapsed_time(e1) / a.reps)
for v in order:
    print(f"{v}: median {statistics.median(times[v]) * 1e3:.1f} us per call ({B} x {a.seconds:g} s)")
