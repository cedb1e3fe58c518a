"""Interleaved A/B of the PESQ front end across library variants in ONE process (GPU box):
every variant's fsem_pesq_front_y10_f32 (the joint front end, as bench.py's roofline times it)
is launched `--reps` times per round on the same inputs, HIP-event timed on the current stream,
over `--rounds` rounds in rotating order; prints the median per variant and whether its Bark
bands and powers are bitwise those of the first variant.

    python tools/ab_front.py va vb ...     (libraries fast_speech_enhancement_metrics_amd/lib/var/NAME.so)
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
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--reps", type=int, default=4)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--joint", type=int, default=1)
a = ap.parse_args()

libs = {}
for v in a.variants:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "fast_speech_enhancement_metrics_amd", "lib",
                                   "var", v + ".so"), mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _native.SIGNATURES.items():
        if hasattr(lib, name):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    libs[v] = lib

B, L = a.batch, a.length
c, n, _ = speech_like_pairs(B, L, 16000, seed=42, device="cuda")
dev = c.device
lib0 = next(iter(libs.values()))
F = lib0.fsem_pesq_frames(L)
bark = torch.empty(2 * B, 49, (F + 31) // 32 * 32, device=dev)
power = torch.empty(2 * B, device=dev)
ws = _native.workspace(max(l.fsem_pesq_front_workspace_bytes(B, L) for l in libs.values()), dev)
y_ld = ((5 * L + 7) // 8 + 63) // 64 * 64
y10 = torch.empty(2 * B, y_ld, device=dev)
v_ld = (((5 * L + 7) // 8) // 64 + 1 + 63) // 64 * 64
vad = torch.empty(B, v_ld, 2, device=dev)
h = torch.cuda.current_stream().cuda_stream


def launch(lib):
    if a.joint:
        rc = lib.fsem_pesq_front_y10_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, bark.data_ptr(), power.data_ptr(),
                                         y10.data_ptr(), y_ld, vad.data_ptr(), v_ld, ws.data_ptr(), ws.numel(), h)
    else:
        rc = lib.fsem_pesq_front_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, bark.data_ptr(), power.data_ptr(),
                                     ws.data_ptr(), ws.numel(), h)
    assert rc == 0, rc


times = {v: [] for v in libs}
for v, lib in libs.items():  # warm-up
    for _ in range(2):
        launch(lib)
torch.cuda.synchronize()
order = list(libs)
for r in range(a.rounds):
    for v in order[r % len(order):] + order[:r % len(order)]:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            launch(libs[v])
        e1.record()
        e1.synchronize()
        times[v].append(e0.elapsed_time(e1) / a.reps)
outs = {}
for v in libs:  # outputs of each variant (the same inputs): bitwise comparison with the first
    launch(libs[v])
    torch.cuda.synchronize()
    outs[v] = (bark.clone(), power.clone())
first = next(iter(outs))
for v in libs:
    t = times[v]
    same = all(torch.equal(a, b) for a, b in zip(outs[v], outs[first]))
    print(f"{v}: median {statistics.median(t):.4f} ms  min {min(t):.4f}  max {max(t):.4f}  ({len(t)} rounds)"
          f"  bark/power bitwise equal to {first}: {same}")
