"""Host cost of launching one call (no host sync): the raw C-ABI entry with preallocated buffers,
the scores() method, and a trivial ctypes call for scale.

    python tools/probes/launch_cost.py [--batch 64] [--seconds 16]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI, _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--seconds", type=float, default=16.0)
ap.add_argument("--reps", type=int, default=100)
a = ap.parse_args()
B, L = a.batch, int(a.seconds * 16000)
c, n, _ = speech_like_pairs(B, L, 16000, device="cuda")
lib = _native.load()
out = torch.empty(3, B, device="cuda")
ws = _native.workspace(lib.fsem_pesq_stoi_workspace_bytes(B, L), "cuda")
wsp = _native.workspace(lib.fsem_pesq_workspace_bytes(B, L), "cuda")
wss = _native.workspace(lib.fsem_stoi_workspace_bytes(B, L, 16000), "cuda")
h = torch.cuda.current_stream().cuda_stream


def per_call(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return 1e6 * (t1 - t0) / a.reps


res = {
    "ctypes trivial (fsem_pesq_frames)": per_call(lambda: lib.fsem_pesq_frames(L)),
    "workspace query": per_call(lambda: lib.fsem_pesq_stoi_workspace_bytes(B, L)),
    "torch.empty workspace": per_call(lambda: _native.workspace(lib.fsem_pesq_stoi_workspace_bytes(B, L), "cuda")),
    "fsem_pesq_stoi_f32": per_call(lambda: lib.fsem_pesq_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, L, None,
                                                                 out[0].data_ptr(), out[1].data_ptr(),
                                                                 out[2].data_ptr(), ws.data_ptr(), ws.numel(), h)),
    "fsem_pesq_wb_f32": per_call(lambda: lib.fsem_pesq_wb_f32(c.data_ptr(), n.data_ptr(), B, L, L, None,
                                                             out[0].data_ptr(), wsp.data_ptr(), wsp.numel(), h)),
    "fsem_stoi_f32": per_call(lambda: lib.fsem_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, 16000,
                                                       out[1].data_ptr(), out[2].data_ptr(), wss.data_ptr(),
                                                       wss.numel(), h)),
}
jt, p, s = PESQ_STOI(16000, use_gpu=True), PESQ(16000, use_gpu=True), STOI(16000, use_gpu=True)
res["PESQ_STOI.scores"] = per_call(lambda: jt.scores(c, n))
res["PESQ.scores"] = per_call(lambda: p.scores(c, n))
res["STOI.scores"] = per_call(lambda: s.scores(c, n, 16000))
for k, v in res.items():
    print(f"{k:40s} {v:8.1f} us/call")
