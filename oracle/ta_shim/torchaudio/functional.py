"""ORACLE ONLY: torchaudio.functional.lfilter / resample restatements (torchaudio 2.8.0)."""
import numpy as np
import torch

from oracle import ta as _ta


def lfilter(waveform, a_coeffs, b_coeffs, clamp: bool = True, batching: bool = True):
    """torchaudio 2.8 ``lfilter`` for 1-D coefficient vectors.

    FIR part exactly as torchaudio: left-pad by order-1, conv1d with flipped b, divide
    by a0; IIR part: the sequential fp32 loop (oracle/c/lfilter_f32.c).

    ``FSEM_SHIM_FIR=f64`` (sensitivity studies only, tests/golden/make_golden.py): the FIR part
    accumulated in float64 and rounded once -- another admissible float32 evaluation order of
    the same filter, to show where the reference's own result depends on summation order.
    """
    import os
    assert a_coeffs.ndim == 1 and b_coeffs.ndim == 1
    shape = waveform.shape
    x = waveform.reshape(-1, 1, shape[-1]).to(torch.float32)
    order = a_coeffs.shape[0]
    xp = torch.nn.functional.pad(x, [order - 1, 0])
    bflip = b_coeffs.flip(0).to(torch.float32).view(1, 1, -1)
    if os.environ.get("FSEM_SHIM_FIR") == "f64":
        w = torch.nn.functional.conv1d(xp.double(), bflip.double()).to(torch.float32)
    else:
        w = torch.nn.functional.conv1d(xp, bflip)
    w = w / a_coeffs[0]
    y = _ta.lfilter_iir(w.reshape(-1, shape[-1]).cpu().numpy(), a_coeffs.cpu().numpy())
    out = torch.from_numpy(y).reshape(shape).to(waveform.device)
    if clamp:
        out = torch.clamp(out, min=-1.0, max=1.0)
    return out


def resample(waveform, orig_freq, new_freq, **kw):
    from .transforms import Resample
    return Resample(orig_freq, new_freq)(waveform)
