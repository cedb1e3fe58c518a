"""GPU-box diagnostic: the engine's 1/3-octave envelopes (fsem_stoi_tob_f32) and STOI / ESTOI of
given 10 kHz pairs, saved for a CPU-side comparison with the oracle's float64 envelopes.

    python tools/probes/tob_dump.py OUT.npz [golden_name ...]     (default: tone_probe_10k)

Golden fixtures at other rates are resampled to 10 kHz on the GPU first (fsem_resample_f32)."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(HERE))

from fast_speech_enhancement_metrics_amd import STOI, _native  # noqa: E402
from tests.conftest import load_golden  # noqa: E402


def tob_of(c, n):
    lib = _native.load()
    B, L = c.shape
    NV = (L - 256) // 128 + 1
    tmax = NV - 2
    kept = torch.empty(B, dtype=torch.int32, device=c.device)
    tob = torch.zeros(2 * B, 15, tmax, device=c.device)
    ws = _native.workspace(lib.fsem_stoi_workspace_bytes(B, L, 10000), c.device)
    _native.check(lib.fsem_stoi_tob_f32(c.data_ptr(), n.data_ptr(), B, L, L, kept.data_ptr(), tob.data_ptr(), tmax,
                                        ws.data_ptr(), ws.numel(), _native.stream_handle(c.device)), "tob")
    torch.cuda.synchronize()
    return kept.cpu().numpy(), tob.cpu().numpy()


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or ["tone_probe_10k"]
    res = {}
    for name in names:
        if ":" in name:  # edges_16k:<case>: the edge input as make_golden.py built it
            from tests.conftest import edge_inputs
            gname, case = name.split(":")
            g = load_golden(gname)
            c, n = (t.cuda() for t in edge_inputs(g, case))
        else:
            g = load_golden(name)
            c = torch.from_numpy(g["clean_f"]).cuda()
            n = torch.from_numpy(g["noisy_f"]).cuda()
        sr = int(g.get("sample_rate", 10000))
        if sr != 10000:
            from fast_speech_enhancement_metrics_amd.base import resample_rows
            c, n, _ = resample_rows(c, n, None, sr, 10000)
            c, n = c.contiguous(), n.contiguous()
        kept, tob = tob_of(c, n)
        s, e = STOI(10000, use_gpu=True).scores(c, n)
        name = name.replace(":", "__")
        res[name + "_kept"] = kept
        res[name + "_tob"] = tob
        res[name + "_stoi"] = s.cpu().numpy()
        res[name + "_estoi"] = e.cpu().numpy()
        res[name + "_x10_clean"] = c.cpu().numpy()
        res[name + "_x10_noisy"] = n.cpu().numpy()
        print(name, "stoi", res[name + "_stoi"], "estoi", res[name + "_estoi"], flush=True)
    np.savez_compressed(out, **res)


if __name__ == "__main__":
    main()
