"""Power spectrogram module of the PESQ stage API (the reference's ``PESQ.to_spec``, a
``torchaudio.transforms.Spectrogram``, PESQ.py:63-71).  torchaudio is not part of this build:
this is its published transform -- ``torch.stft`` with the given window, |X|^power -- for the
arguments the reference uses.  The engine's own framing + FFT lives in ``pesq_front``.
"""
from __future__ import annotations

from typing import Callable

import torch


class Spectrogram(torch.nn.Module):
    def __init__(self, n_fft: int = 400, win_length: int | None = None, hop_length: int | None = None,
                 pad: int = 0, window_fn: Callable[..., torch.Tensor] = torch.hann_window,
                 power: float | None = 2.0, normalized: bool = False, center: bool = True,
                 pad_mode: str = "reflect", onesided: bool = True):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        self.pad = pad
        self.power = power
        self.normalized = normalized
        self.center = center
        self.pad_mode = pad_mode
        self.onesided = onesided
        self.register_buffer("window", window_fn(self.win_length), persistent=False)

    def forward(self, waveform: torch.Tensor) -> torch.Tensor:
        """[..., time] -> [..., n_fft // 2 + 1, frames] (power spectrum for power = 2)."""
        shape = waveform.shape
        x = waveform.reshape(-1, shape[-1])
        if self.pad:
            x = torch.nn.functional.pad(x, (self.pad, self.pad))
        spec = torch.stft(x, n_fft=self.n_fft, hop_length=self.hop_length, win_length=self.win_length,
                          window=self.window.to(device=x.device, dtype=x.dtype), center=self.center,
                          pad_mode=self.pad_mode, normalized=False, onesided=self.onesided, return_complex=True)
        if self.normalized:
            spec = spec / self.window.pow(2.0).sum().sqrt()
        if self.power is not None:
            spec = spec.abs().pow(self.power) if self.power != 1.0 else spec.abs()
        return spec.reshape(shape[:-1] + spec.shape[-2:])
