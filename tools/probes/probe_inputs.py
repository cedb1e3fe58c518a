"""Input-form probe of the drop-in API on the GPU: dtypes, non-contiguous views, NaN / Inf
samples, zero / one-sample ragged rows -- scores next to the float32 contiguous result.

    python tools/probes/probe_inputs.py
"""
import os
import sys
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI  # noqa: E402
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs  # noqa: E402

warnings.simplefilter("ignore")
c, n, _ = speech_like_pairs(3, 48000, 16000, seed=5, device="cuda")
m = PESQ_STOI(16000, use_gpu=True)


def show(name, fn):
    try:
        r = fn()
        print(f"{name:28s}", [(round(d['PESQ'], 4), round(d['STOI'], 4), round(d['ESTOI'], 4)) for d in r])
    except Exception as ex:  # noqa: BLE001
        print(f"{name:28s} raised {type(ex).__name__}: {ex}")


show("float32", lambda: m(c, n))
show("float64", lambda: m(c.double(), n.double()))
show("float16", lambda: m(c.half(), n.half()))
show("bfloat16", lambda: m(c.bfloat16(), n.bfloat16()))
show("cpu tensors", lambda: m(c.cpu(), n.cpu()))
show("numpy arrays", lambda: m(c.cpu().numpy(), n.cpu().numpy()))
t = torch.stack([c, n], 2)  # [B, L, 2]: strided rows
show("strided views", lambda: m(t[:, :, 0], t[:, :, 1]))
show("transposed T view", lambda: m(c.t().contiguous().t(), n.t().contiguous().t()))
nn = n.clone(); nn[1, 1000] = float("nan")
show("NaN in denoised row 1", lambda: m(c, nn))
nn = n.clone(); nn[2, 2000] = float("inf")
show("Inf in denoised row 2", lambda: m(c, nn))
cc = c.clone(); cc[0, 5] = float("nan")
show("NaN in clean row 0", lambda: m(cc, n))
show("ragged 0 / 1 / full", lambda: m(c, n, lengths=[0, 1, 48000]))
show("1-D pair", lambda: m(c[0], n[0]))
show("PESQ only", lambda: [dict(PESQ=d["PESQ"], STOI=0, ESTOI=0) for d in PESQ(16000, use_gpu=True)(c, n)])
show("STOI only", lambda: [dict(PESQ=0, **d) for d in STOI(16000, use_gpu=True)(c, n)])

# NaN / Inf rows against the oracle (reference semantics: NaN propagates where the sample is used)
from oracle import pesq_oracle, stoi_oracle  # noqa: E402
for name, (cc, nn) in {"NaN denoised": (c, n.clone().index_put_((torch.tensor([1]), torch.tensor([1000])), torch.tensor(float("nan"), device="cuda"))),
                       "Inf denoised": (c, n.clone().index_put_((torch.tensor([2]), torch.tensor([2000])), torch.tensor(float("inf"), device="cuda"))),
                       "Inf denoised mid": (c, n.clone().index_put_((torch.tensor([2]), torch.tensor([24000])), torch.tensor(float("inf"), device="cuda"))),
                       "NaN clean": (c.clone().index_put_((torch.tensor([0]), torch.tensor([5])), torch.tensor(float("nan"), device="cuda")), n)}.items():
    r = m(cc, nn)
    a, b = cc.cpu().numpy(), nn.cpu().numpy()
    op = pesq_oracle.pesq(a, b)
    try:
        os_, oe = stoi_oracle.stoi(a, b, 16000)
    except Exception as ex:  # noqa: BLE001
        os_ = oe = [f"raised {type(ex).__name__}"] * 3
    print(f"{name:18s} gpu", [(round(d['PESQ'], 4), round(d['STOI'], 4), round(d['ESTOI'], 4)) for d in r])
    print(f"{'':18s} oracle", [(round(float(x), 4) if not isinstance(x, str) else x, y, z) for x, y, z in zip(op, np.round(os_, 4) if not isinstance(os_[0], str) else os_, np.round(oe, 4) if not isinstance(oe[0], str) else oe)])
