"""Does the joint engine gain from running consecutive row chunks on two streams (chunk k+1's
front end beside chunk k's STOI tail and PESQ back end)?  Times N chunks of `--chunk` rows of
10 s pairs through fsem_pesq_stoi_f32: all on one stream (serial) against alternating streams
with separate workspaces (overlapped), interleaved rounds, and checks the scores are equal.

    python tools/probes/ab_overlap.py [--chunk 2048] [--chunks 4] [--rounds 6]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--chunk", type=int, default=2048)
ap.add_argument("--chunks", type=int, default=4)
ap.add_argument("--rounds", type=int, default=6)
ap.add_argument("--length", type=int, default=160000)
a = ap.parse_args()

lib = _native.load()
dev = torch.device("cuda:0")
C, N, L = a.chunk, a.chunks, a.length
c, n, _ = speech_like_pairs(C * N, L, 16000, seed=3, device=dev)
wsb = lib.fsem_pesq_stoi_workspace_bytes(C, L)
ws = [_native.workspace(wsb, dev), torch.empty(wsb, dtype=torch.uint8, device=dev)]
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
outs = {m: torch.empty(3, C * N, device=dev) for m in ("serial", "overlap")}


def run(mode):
    s0 = streams[0]
    start = torch.cuda.Event(enable_timing=True)
    start.record(s0)
    if mode == "overlap":
        streams[1].wait_stream(s0)
    for k in range(N):
        i = k % 2 if mode == "overlap" else 0
        st = streams[i]
        o = outs[mode]
        lo = k * C
        with torch.cuda.stream(st):
            rc = lib.fsem_pesq_stoi_f32(c[lo].data_ptr(), n[lo].data_ptr(), C, L, L, None, o[0, lo:].data_ptr(),
                                        o[1, lo:].data_ptr(), o[2, lo:].data_ptr(), ws[i].data_ptr(), wsb,
                                        st.cuda_stream)
        assert rc == 0, rc
    if mode == "overlap":
        s0.wait_stream(streams[1])
    end = torch.cuda.Event(enable_timing=True)
    end.record(s0)
    end.synchronize()
    return start.elapsed_time(end)


for m in outs:  # warm-up
    run(m)
t = {m: [] for m in outs}
for r in range(a.rounds):
    for m in (("serial", "overlap") if r % 2 == 0 else ("overlap", "serial")):
        t[m].append(run(m))
for m in outs:
    med = statistics.median(t[m])
    print(f"{m}: median {med:.3f} ms for {N} x {C} rows ({med / N:.3f} ms per chunk, "
          f"{C * N / med * 1e3:,.0f} utt/s)  min {min(t[m]):.3f} max {max(t[m]):.3f}")
print("scores equal:", torch.equal(outs["serial"], outs["overlap"]))
