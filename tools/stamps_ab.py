"""Per-phase cycles of pesq_front<joint> for several diagnostic (FSEM_STAMPS) library variants,
each driven through its own fsem_pesq_stoi_f32 (so variants of other rounds, whose ABI lacks
later entries, load too).  Prints the mean s_memtime ticks per phase of one item (the last item
of each persistent block); compare variants phase by phase -- never quote a stamp build's time.

    EXTRA=-DFSEM_STAMPS bash tools/build_variant.sh stamps_X <rev>
    python tools/stamps_ab.py stamps_X stamps_Y
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
from fast_speech_enhancement_metrics_amd import _native  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

B, L = int(os.environ.get("B", "4096")), 160000
c, n, _ = speech_like_pairs(B, L, 16000, seed=42, device="cuda")
_vp, _i64, _sz = ctypes.c_void_p, ctypes.c_int64, ctypes.c_size_t
SEGS = [("tile->LDS", 0, 14), ("resample", 14, 1), ("IIR pass1", 1, 2), ("scan", 2, 3), ("IIR pass2", 3, 4),
        ("FFT rounds", 4, 13), ("bark", 13, 15)]
rows = {}
for v in sys.argv[1:]:
    lib = ctypes.CDLL(os.path.join(os.path.dirname(__file__), "..", "fast_speech_enhancement_metrics_amd", "lib",
                                   "var", v + ".so"), mode=ctypes.RTLD_LOCAL)
    lib.fsem_pesq_stoi_workspace_bytes.restype = _sz
    lib.fsem_pesq_stoi_workspace_bytes.argtypes = [_i64, _i64]
    lib.fsem_pesq_stoi_f32.argtypes = [_vp, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]
    lib.fsem_debug_read_stamps.argtypes = [_vp, _sz]
    ws = _native.workspace(lib.fsem_pesq_stoi_workspace_bytes(B, L), c.device)
    out = torch.empty(3, B, device=c.device)
    for _ in range(3):
        rc = lib.fsem_pesq_stoi_f32(c.data_ptr(), n.data_ptr(), B, L, L, None, out[0].data_ptr(), out[1].data_ptr(),
                                    out[2].data_ptr(), ws.data_ptr(), ws.numel(),
                                    torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
    torch.cuda.synchronize()
    buf = np.zeros((65536, 16), dtype=np.uint64)
    assert lib.fsem_debug_read_stamps(buf.ctypes.data, buf.nbytes) == 0
    st = buf.astype(np.float64)
    valid = (st[:, 15] > 0) & (st[:, 0] > 0) & (st[:, 15] > st[:, 0])
    tot = (st[valid, 15] - st[valid, 0]).mean()
    r = {"item": tot}
    for nm, a, b in SEGS:
        ok = valid & (st[:, a] > 0) & (st[:, b] > 0) & (st[:, b] >= st[:, a])
        r[nm] = (st[ok, b] - st[ok, a]).mean() if ok.any() else float("nan")
    rows[v] = r
    del ws
names = list(rows)
print(f"{'phase':16s}" + "".join(f"{v:>14s}" for v in names))
for key in ["item"] + [s[0] for s in SEGS]:
    print(f"{key:16s}" + "".join(f"{rows[v][key]:14.0f}" for v in names))
