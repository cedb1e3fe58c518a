"""ORACLE ONLY: torchaudio.transforms.Resample / Spectrogram restatements (torchaudio 2.8.0)."""
import math

import torch

from oracle import ta as _ta


class Resample(torch.nn.Module):
    """``Resample(orig, new)``: sinc_interp_hann kernel (width 6, rolloff 0.99), applied
    with the same pad + strided conv1d + interleave + ceil-truncate as torchaudio."""

    def __init__(self, orig_freq=16000, new_freq=16000, **kw):
        super().__init__()
        self.orig_freq = orig_freq
        self.new_freq = new_freq
        if orig_freq != new_freq:
            kern, self.width, self.orig, self.new = _ta.sinc_resample_kernel(orig_freq, new_freq)
            self.register_buffer("kernel", torch.from_numpy(kern).unsqueeze(1))

    def forward(self, waveform):
        if self.orig_freq == self.new_freq:
            return waveform
        shape = waveform.size()
        w = waveform.reshape(-1, shape[-1])
        n = w.shape[1]
        w = torch.nn.functional.pad(w, (self.width, self.width + self.orig))
        res = torch.nn.functional.conv1d(w[:, None], self.kernel.to(w.device), stride=self.orig)
        res = res.transpose(1, 2).reshape(w.shape[0], -1)
        target = int(math.ceil(self.new * n / self.orig))
        res = res[..., :target]
        return res.view(shape[:-1] + res.shape[-1:])


class Spectrogram(torch.nn.Module):
    """``Spectrogram(..., power=2, center=False)`` = torch.stft(...).abs().pow(2)."""

    def __init__(self, n_fft=400, win_length=None, hop_length=None, pad=0,
                 window_fn=torch.hann_window, power=2.0, normalized=False, wkwargs=None,
                 center=True, pad_mode="reflect", onesided=True, return_complex=None):
        super().__init__()
        self.n_fft = n_fft
        self.win_length = win_length if win_length is not None else n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 2
        window = window_fn(self.win_length) if wkwargs is None else window_fn(self.win_length, **wkwargs)
        self.register_buffer("window", window)
        self.power = power
        self.center = center
        self.pad_mode = pad_mode
        self.onesided = onesided
        assert pad == 0 and not normalized

    def forward(self, waveform):
        shape = waveform.size()
        w = waveform.reshape(-1, shape[-1])
        spec = torch.stft(w, n_fft=self.n_fft, hop_length=self.hop_length, win_length=self.win_length,
                          window=self.window.to(w.device), center=self.center, pad_mode=self.pad_mode,
                          normalized=False, onesided=self.onesided, return_complex=True)
        spec = spec.reshape(shape[:-1] + spec.shape[-2:])
        if self.power is None:
            return spec
        if self.power == 1.0:
            return spec.abs()
        return spec.abs().pow(self.power)
