"""Resampler of BaseMetric.prepare_audio (reference fast_se_metrics/base.py:13,19-20).

Same result as ``torchaudio.transforms.Resample(orig, new)`` with its defaults
(sinc_interp_hann, lowpass_filter_width 6, rolloff 0.99): the kernel formula is
torchaudio 2.8's ``_get_sinc_resample_kernel`` (float64 build, float32 phase offsets).
On CUDA tensors the work runs in libfsem (``fsem_resample_f32``); on CPU tensors it is a
strided ``conv1d`` (the reference's own CPU behaviour).
"""
from __future__ import annotations

import math

import torch

from . import _native


def sinc_kernel(orig_freq: int, new_freq: int, width_taps: int = 6, rolloff: float = 0.99):
    g = math.gcd(int(orig_freq), int(new_freq))
    orig, new = int(orig_freq) // g, int(new_freq) // g
    base = min(orig, new) * rolloff
    width = math.ceil(width_taps * orig / base)
    idx = torch.arange(-width, width + orig, dtype=torch.float64)[None, :] / orig
    phase = (torch.arange(0, -new, -1)[:, None] / new).to(torch.float64)  # int / int -> float32, as torchaudio
    t = (phase + idx) * base
    t = t.clamp(-width_taps, width_taps)
    window = torch.cos(t * math.pi / width_taps / 2) ** 2
    t = t * math.pi
    kern = torch.where(t == 0, torch.ones_like(t), t.sin() / t) * (window * (base / orig))
    return kern.to(torch.float32), width, orig, new


class Resample(torch.nn.Module):
    def __init__(self, orig_freq: int = 16000, new_freq: int = 16000):
        super().__init__()
        self.orig_freq = int(orig_freq)
        self.new_freq = int(new_freq)
        if self.orig_freq != self.new_freq:
            kern, self.width, self.orig, self.new = sinc_kernel(self.orig_freq, self.new_freq)
            self.register_buffer("kernel", kern.unsqueeze(1), persistent=False)

    def output_length(self, n: int) -> int:
        if self.orig_freq == self.new_freq:
            return n
        return int(math.ceil(self.new * n / self.orig))

    def forward(self, waveform: torch.Tensor, lengths: torch.Tensor | None = None) -> torch.Tensor:
        """[..., n] -> [..., ceil(new * n / orig)].  ``lengths`` ([rows] ints, rows = the flattened
        leading dims): row r is resampled as its first lengths[r] samples alone (zeros past them)
        and its output past ceil(new * lengths[r] / orig) is zero -- the zero-padded ragged rows of
        BaseMetric.__call__ without materialising them."""
        if self.orig_freq == self.new_freq:
            return waveform
        shape = waveform.shape
        x = waveform.reshape(-1, shape[-1])
        n = x.shape[1]
        if x.is_cuda:
            x = x.to(torch.float32).contiguous()
            lib = _native.load()
            n_out = self.output_length(n)
            out = torch.empty(x.shape[0], n_out, dtype=torch.float32, device=x.device)
            if x.shape[0] and n:
                st = _native.stream_handle(x.device)
                if lengths is None:
                    rc = lib.fsem_resample_f32(x.data_ptr(), x.shape[0], n, n, out.data_ptr(), n_out,
                                               self.orig_freq, self.new_freq, st)
                else:
                    from .base import device_lengths
                    lens = device_lengths(lengths, x.shape[0], n, x.device)
                    rc = lib.fsem_resample_rows_f32(x.data_ptr(), x.shape[0], n, n, lens.data_ptr(),
                                                    out.data_ptr(), n_out, self.orig_freq, self.new_freq, st)
                _native.check(rc, "resample")
            return out.reshape(shape[:-1] + (n_out,))
        if lengths is not None:
            from .base import zero_tail
            x = zero_tail(x, torch.as_tensor(lengths).reshape(-1))
            res = self.forward(x)
            t = torch.arange(res.shape[-1])
            keep = t[None, :] < torch.as_tensor(
                [self.output_length(int(v)) for v in torch.as_tensor(lengths).reshape(-1).tolist()])[:, None]
            return torch.where(keep, res, torch.zeros((), dtype=res.dtype)).reshape(shape[:-1] + res.shape[-1:])
        xp = torch.nn.functional.pad(x.to(torch.float32), (self.width, self.width + self.orig))
        res = torch.nn.functional.conv1d(xp[:, None], self.kernel.to(xp.device), stride=self.orig)
        res = res.transpose(1, 2).reshape(x.shape[0], -1)[:, :self.output_length(n)]
        return res.reshape(shape[:-1] + res.shape[-1:])
