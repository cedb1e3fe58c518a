"""Interleaved A/B of the whole joint engine call (fsem_pesq_stoi_f32: PESQ-wb + STOI/ESTOI, the
bench's GPU work) across library variants in ONE process on the GPU box: each variant is called
`--reps` times per round on the same device inputs, HIP-event timed on the current stream, over
`--rounds` rounds in rotating order; prints the median per variant and checks that every variant
returns finite scores of the same shape.  Box-to-box spread (clocks, HBM) cancels out of the
comparison, unlike separate bench runs.

    bash tools/build_variant.sh r1 <rev1>; bash tools/build_variant.sh r2 <rev2>; ...
    python tools/ab_joint.py r1 r2 r3        (libraries fast_speech_enhancement_metrics_amd/lib/var/NAME.so)
"""
import argparse
import ctypes
import json
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
ap.add_argument("--rounds", type=int, default=8)
a = ap.parse_args()

_vp, _i64, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
libs = {}
for v in a.variants:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "fast_speech_enhancement_metrics_amd", "lib",
                                   "var", v + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.fsem_pesq_stoi_workspace_bytes.restype = _sz
    lib.fsem_pesq_stoi_workspace_bytes.argtypes = [_i64, _i64]
    lib.fsem_pesq_stoi_f32.restype = ctypes.c_int
    lib.fsem_pesq_stoi_f32.argtypes = [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]
    libs[v] = lib

B, L = a.batch, a.length
c, n, _ = speech_like_pairs(B, L, 16000, seed=42, device="cuda")
dev = c.device
ws = _native.workspace(max(lib.fsem_pesq_stoi_workspace_bytes(B, L) for lib in libs.values()), dev)
outs = {v: torch.empty(3, B, device=dev) for v in libs}
h = torch.cuda.current_stream().cuda_stream


def launch(v):
    o = outs[v]
    rc = libs[v].fsem_pesq_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, o[0].data_ptr(), o[1].data_ptr(),
                                    o[2].data_ptr(), ws.data_ptr(), ws.numel(), h)
    assert rc == 0, (v, rc)


for v in libs:  # warm-up
    for _ in range(2):
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
res = {}
ref = outs[order[0]].cpu()
for v in libs:
    t = times[v]
    o = outs[v].cpu()
    assert torch.isfinite(o).all(), v
    res[v] = {"median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4), "max_ms": round(max(t), 4),
              "max_abs_diff_vs_" + order[0]: [float((o[i] - ref[i]).abs().max()) for i in range(3)]}
    print(f"{v}: median {statistics.median(t):.4f} ms  min {min(t):.4f}  max {max(t):.4f}  ({len(t)} rounds)")
print(json.dumps({"batch": B, "length": L, "reps": a.reps, "rounds": a.rounds, "variants": res}))
