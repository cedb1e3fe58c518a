"""Host-side time of the drop-in call's fast path (joint.py PESQ_STOI._fast_call), piece by piece,
on the bench's 4096 x 10 s batch: Python before the engine call, the C-ABI call itself (argument
conversion + the C++ enqueue), the list allocation, the wait for the GPU and the fill -- each a
median over back-to-back calls, so the pieces that run while the GPU idles between calls show.

    python tools/probes/host_gap.py [--calls 30]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ_STOI, _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.joint import _KEYS  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--length", type=int, default=160000)
ap.add_argument("--calls", type=int, default=30)
a = ap.parse_args()
c, n, _ = speech_like_pairs(a.batch, a.length, 16000, seed=42, device="cuda")
m = PESQ_STOI(16000, use_gpu=True)
for _ in range(5):
    m(c, n)
torch.cuda.synchronize()
lib = _native.load()
pieces = {k: [] for k in ("checks", "slot+ws", "engine_call", "alloc", "wait", "fill", "total", "call_gap")}
prev_end = None
for _ in range(a.calls):
    t0 = time.perf_counter()
    ok = m._fast_ok(c, n)
    B, L = n.shape
    dev = n.device
    stream = torch.cuda.current_stream(dev)
    wsb = m._ws_bytes[(B, L)]
    t1 = time.perf_counter()
    slot = _native.mapped_host_slot(m, 3 * B)
    o = slot[0].data_ptr()
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    t2 = time.perf_counter()
    rc = lib.fsem_pesq_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, c.stride(0), None, o, o + 4 * B, o + 8 * B,
                                ws.data_ptr(), wsb, stream.cuda_stream)
    t3 = time.perf_counter()
    _, pin_np, ev = slot
    ev.record(stream)
    m._held_list = None
    res, h = _native.score_list_alloc(B, _KEYS)
    t4 = time.perf_counter()
    ev.synchronize()
    t5 = time.perf_counter()
    _native.score_list_fill(h, 0, pin_np[:3 * B].reshape(3, B), _KEYS)
    m._held_list = h
    t6 = time.perf_counter()
    assert ok and rc == 0
    for k, v in zip(("checks", "slot+ws", "engine_call", "alloc", "wait", "fill", "total"),
                    (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t6 - t0)):
        pieces[k].append(v * 1e6)
    if prev_end is not None:
        pieces["call_gap"].append((t0 - prev_end) * 1e6)
    del res
    prev_end = time.perf_counter()
for k, v in pieces.items():
    print(f"{k:12s} median {statistics.median(v):9.1f} us   min {min(v):9.1f}")
# the real call, end to end, for comparison
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.calls):
    m(c, n)
torch.cuda.synchronize()
print(f"drop-in call {(time.perf_counter() - t0) / a.calls * 1e3:.4f} ms per call")
