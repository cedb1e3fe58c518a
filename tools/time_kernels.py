"""Time the PESQ front-end and the STOI pipeline of the library named by FSEM_LIB (A/B builds).

    FSEM_LIB=path/to/variant.so python tools/time_kernels.py [--reps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import PESQ, STOI, _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--batch", type=int, default=4096)
a = ap.parse_args()
lib = _native.load()
B, L = a.batch, 160000
c, n, _ = speech_like_pairs(B, L, device="cuda")
F = lib.fsem_pesq_frames(L)
bark = torch.empty(2 * B, 49, (F + 31) // 32 * 32, device="cuda")
power = torch.empty(2 * B, device="cuda")
ws = _native.workspace(lib.fsem_pesq_front_workspace_bytes(B, L), "cuda")
h = torch.cuda.current_stream().cuda_stream


def front():
    _native.check(lib.fsem_pesq_front_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, bark.data_ptr(), power.data_ptr(),
                                          ws.data_ptr(), ws.numel(), h), "front")


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


from fast_speech_enhancement_metrics_amd import PESQ_STOI  # noqa: E402
p, st = PESQ(16000, use_gpu=True), STOI(16000, use_gpu=True)
jt = PESQ_STOI(16000, use_gpu=True) if hasattr(lib, "fsem_pesq_stoi_f32") else None
t_joint = timeit(lambda: jt.scores(c, n)) if jt is not None else float("nan")
t_front = timeit(front)
t_pesq = timeit(lambda: p.scores(c, n))
t_stoi = timeit(lambda: st.scores(c, n, 16000))
mos = p.scores(c, n)[:4].tolist()
# the back end alone, on the front's outputs
front()
mos_b = torch.empty(B, device="cuda")
wsb = _native.workspace(lib.fsem_pesq_back_workspace_bytes(B, L), "cuda")


def back():
    _native.check(lib.fsem_pesq_back_f32(bark.data_ptr(), power.data_ptr(), B, L, None, mos_b.data_ptr(),
                                         wsb.data_ptr(), wsb.numel(), h), "back")


t_back = timeit(back)
print(f"{os.path.basename(_native.LIB_PATH)}: pesq_front {t_front:.3f} ms  pesq_back {t_back:.3f} ms  PESQ {t_pesq:.3f} ms  "
      f"STOI {t_stoi:.3f} ms  joint {t_joint:.3f} ms  mos[:4] {mos}")
