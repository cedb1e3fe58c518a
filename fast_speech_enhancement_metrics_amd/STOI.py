"""STOI / ESTOI metric -- drop-in for the reference's ``fast_se_metrics.STOI`` (STOI.py:7-205).

Runs at 10 kHz internally (STOI.py:9).  ``use_gpu=True``: libfsem's gfx950 kernels
(``fsem_stoi_f32``) with the 16 -> 10 kHz resampler fused into them (the reference
resamples in BaseMetric.prepare_audio, base.py:19-20; same arithmetic), one device->host
copy of the scores.  ``use_gpu=False``: the package's CPU implementation.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from . import _cpu, _native
from .base import BaseMetric, as_rows, check_row_rate, device_lengths, noisy_shape, same_device, zero_tail
from .batching import resampled_lengths


class STOI(BaseMetric):
    higher_is_better = True
    EXPECTED_SAMPLING_RATE = 10000

    def __init__(self, sample_rate: int = 10000, use_gpu: bool = False, *, devices=None):
        super().__init__(sample_rate, use_gpu, devices=devices)
        self.sampling_frequency = self.EXPECTED_SAMPLING_RATE
        self.win_length = 256
        self.hop_length = self.win_length // 2
        self.n_fft = 512
        self.num_octave_bands = 15
        self.min_frequency = 150
        self.N = 30
        self.beta = -15.0
        self.dynamic_range = 40

    @staticmethod
    def normalize(x: torch.Tensor, dim: int = 0) -> torch.Tensor:
        """In place, as STOI.py:113-119: centre along ``dim`` and divide by the L2 norm, with the
        reference's ``1e-12 * randn`` term taken in expectation (deterministic, as the engine):
        the squared norm gains N * 1e-24 (N = x.shape[dim]) -- no change for any slice with a
        spread above ~1e-8, 0 for a zero-variance slice (the reference: a random unit vector),
        ~0 for a slice far below the noise.  Non-finite slices stay non-finite (NaN / Inf
        propagate as in the reference)."""
        x -= x.mean(dim=dim, keepdim=True)
        x /= torch.sqrt(x.square().sum(dim=dim, keepdim=True) + x.shape[dim] * 1e-24)
        return x

    # ------------------------------------------------------------------ reference attributes
    def get_octave_band_matrix(self) -> torch.Tensor:
        """[15, 257] float32 1/3-octave band matrix (STOI.py:26-47): band i covers the FFT bins
        from the one nearest 150 * 2^((2i - 1) / 6) Hz up to (excluding) the one nearest
        150 * 2^((2i + 1) / 6) Hz."""
        return _cpu._OBM.to(torch.float32).clone()

    @property
    def octave_band_matrix(self) -> torch.Tensor:
        """STOI.py:19, on the metric's device (built on first access)."""
        if getattr(self, "_octave_band_matrix", None) is None:
            self._octave_band_matrix = self.get_octave_band_matrix().to(self.device)
        return self._octave_band_matrix

    @property
    def window(self) -> torch.Tensor:
        """[256] float32 analysis window hann(257)[1:] (STOI.py:24), on the metric's device."""
        if getattr(self, "_window", None) is None:
            self._window = torch.hann_window(self.win_length + 1, dtype=torch.float32, device=self.device)[1:]
        return self._window

    # ------------------------------------------------------------------ stage methods
    # The reference's pipeline stages (STOI.py:49-198) on 10 kHz tensors, as torch expressions on
    # the metric's device (the overlap-add without the reference's per-utterance Python loop).
    # Scores do not go through these: on the GPU compute_metric runs the whole engine
    # (fsem_stoi_f32), which never materialises the overlap-added signal or the [B, S, 15, 30]
    # segments.
    def stft(self, speech: torch.Tensor, lengths: torch.Tensor) -> torch.Tensor:
        """[N, T] -> [N, 257, frames] power spectrogram (n_fft 512, the 256-sample window centred,
        hop 128, center=False); frames at or past 1 + (length - 512) // 128 are zeroed (STOI.py:49-69)."""
        spec = torch.stft(speech, n_fft=self.n_fft, hop_length=self.hop_length, win_length=self.win_length,
                          window=self.window.to(speech.device, speech.dtype), center=False, normalized=False,
                          return_complex=True, onesided=True).abs().square()
        n_valid = 1 + (lengths.to(spec.device) - self.n_fft) // self.hop_length
        t = torch.arange(spec.shape[-1], device=spec.device)
        return spec.masked_fill((t[None, :] >= n_valid[:, None])[:, None, :], 0)

    def overlap_and_add(self, frames: torch.Tensor, lengths: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Kept frames [sum(lengths), 256] of B utterances (``lengths`` frames each, in order) ->
        (signals [B, max_len], (lengths + 1) * 128): frame j of utterance b added at 128 j
        (STOI.py:71-86)."""
        lengths = lengths.to(frames.device)
        out_len = (lengths + 1) * self.hop_length
        B = lengths.numel()
        width = int(out_len.max().item()) if B else 0
        sig = torch.zeros(B, width, dtype=frames.dtype, device=frames.device)
        if frames.numel():
            utt = torch.repeat_interleave(torch.arange(B, device=frames.device), lengths)
            first = torch.cumsum(lengths, 0) - lengths  # index of each utterance's first frame
            j = torch.arange(frames.shape[0], device=frames.device) - first[utt]
            pos = (utt * width + self.hop_length * j)[:, None] + torch.arange(self.win_length, device=frames.device)
            sig.view(-1).index_add_(0, pos.reshape(-1), frames.reshape(-1))
        return sig, out_len

    def remove_silent_frames(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor):
        """Frames (256, hop 128, windowed) more than 40 dB below the clean signal's loudest frame are
        dropped from both signals, which are rebuilt by overlap-add -> (clean, denoised, lengths)
        (STOI.py:88-111)."""
        w = self.window.to(clean_speech.device, clean_speech.dtype)
        cf = clean_speech.unfold(1, self.win_length, self.hop_length) * w
        df = denoised_speech.unfold(1, self.win_length, self.hop_length) * w
        energy = 20 * torch.log10(torch.linalg.vector_norm(cf, dim=2) + 1e-9)
        keep = (energy.amax(dim=1, keepdim=True) - self.dynamic_range - energy) < 0
        n = keep.sum(1)
        c, lens = self.overlap_and_add(cf[keep], n)
        d, _ = self.overlap_and_add(df[keep], n)
        return c, d, lens

    def compute_segments(self, speech: torch.Tensor, lengths: torch.Tensor):
        """1/3-octave band envelopes sqrt(OBM . |STFT|^2) [N, 15, T] cut into the T - 29 sliding
        30-frame windows (views) (STOI.py:121-127)."""
        obm = self.octave_band_matrix.to(speech.device, speech.dtype)
        tob = torch.sqrt(torch.matmul(obm, self.stft(speech, lengths)))
        return [tob[:, :, m:m + self.N] for m in range(max(tob.shape[2] - self.N + 1, 0))]

    def equalize_clip(self, clean_segments: torch.Tensor, denoised_segments: torch.Tensor) -> torch.Tensor:
        """Denoised segments scaled to the clean segments' norm over the 30 frames, then clipped at
        (1 + 10^(-beta/20)) x clean (STOI.py:129-139)."""
        nc = torch.linalg.vector_norm(clean_segments, dim=3, keepdim=True)
        nd = torch.linalg.vector_norm(denoised_segments, dim=3, keepdim=True)
        bound = clean_segments * (1 + 10 ** (-self.beta / 20))
        return torch.minimum(denoised_segments * (nc / (nd + 1e-9)), bound)

    def compute_correlation(self, clean_segments: torch.Tensor, denoised_segments: torch.Tensor,
                            mask: torch.Tensor, extended: bool) -> torch.Tensor:
        """Masked sum over (segment, band, frame) of the products, / 30 (ESTOI) or / 15 (STOI)
        (STOI.py:141-151)."""
        prod = denoised_segments * clean_segments * mask[:, :, None, None]
        return prod.sum(dim=(1, 2, 3)) / (self.N if extended else self.num_octave_bands)

    @torch.no_grad()
    def compute_stoi(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor):
        """(stoi [B], estoi [B]) of 10 kHz signals (STOI.py:153-198); with no 30-frame segment in
        the batch, the reference's warning and (tensor(0), tensor(0)).  GPU: the engine."""
        if clean_speech.is_cuda:
            s, e = self.scores(clean_speech, denoised_speech, self.EXPECTED_SAMPLING_RATE)
        else:
            s, e = _cpu.rows_parallel(_cpu.stoi, torch.atleast_2d(clean_speech), torch.atleast_2d(denoised_speech))
        if bool(torch.isnan(s).all()):
            warnings.warn("Not enough non-silent frames. Please check your sound files", RuntimeWarning, stacklevel=2)
            return torch.tensor(0), torch.tensor(0)
        return s, e

    def scores(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor, sample_rate: int | None = None,
               lengths=None):
        """(stoi[B], estoi[B]) tensors on the metric's device; NaN where no segment exists.

        Rows at ``sample_rate``; None means rows already at 10 kHz, which requires a 10 kHz metric
        (``STOI(16000).scores`` must be told its rows' rate).  ``lengths`` (optional, [B] ints at that rate):
        row b holds lengths[b] samples and scores as the reference would on the unpadded row.
        """
        sr = check_row_rate(self, sample_rate)
        if self.fans_out():
            if noisy_shape(clean_speech) != noisy_shape(denoised_speech):
                raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
            return self.fan_out(lambda c, n, lk: self._rows_scores(c, n, sr, lk), clean_speech, denoised_speech,
                                lengths, 2, balance=lengths)
        return self._rows_scores(clean_speech, denoised_speech, sr, lengths)

    def _rows_scores(self, clean_speech, denoised_speech, sr: int, lengths):
        """(stoi [B], estoi [B]) of rows at rate ``sr`` on their own device (one engine call)."""
        clean = as_rows(clean_speech)
        noisy = as_rows(denoised_speech)
        if noisy.shape != clean.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        same_device(clean, noisy)
        B, L = clean.shape
        if not clean.is_cuda:
            if lengths is not None:
                lens = device_lengths(lengths, B, L, "cpu")
                if sr != self.EXPECTED_SAMPLING_RATE:
                    clean, noisy = self._resample_cpu(zero_tail(clean, lens), sr), self._resample_cpu(zero_tail(noisy, lens), sr)
                    lens = resampled_lengths(lens, sr, self.EXPECTED_SAMPLING_RATE)
                return _cpu.per_row(_cpu.stoi, clean, noisy, lens)
            if sr != self.EXPECTED_SAMPLING_RATE:
                return _cpu.rows_parallel(lambda c, n: _cpu.stoi(self._resample_cpu(c, sr), self._resample_cpu(n, sr)),
                                          clean, noisy)
            return _cpu.rows_parallel(_cpu.stoi, clean, noisy)
        lib = _native.load()
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if clean.stride(0) != noisy.stride(0) or L % 4:
            # rows must be readable up to ceil4(L) floats (include/fsem.h): pad odd lengths
            pad = (-L) % 4
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        s = torch.empty(B, dtype=torch.float32, device=clean.device)
        e = torch.empty(B, dtype=torch.float32, device=clean.device)
        nbytes = lib.fsem_stoi_workspace_bytes(B, L, sr)
        if nbytes == 0:
            raise NotImplementedError(f"unsupported sample rate {sr}: its resampling filter to 10 kHz would be longer "
                                      "than 8192 taps (include/fsem.h, FSEM_ERATE)")
        ws = _native.workspace(nbytes, clean.device)
        rc = lib.fsem_stoi_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                               lens.data_ptr() if lens is not None else None, sr, s.data_ptr(),
                               e.data_ptr(), ws.data_ptr(), ws.numel(), _native.stream_handle(clean.device))
        if rc == _native.FSEM_ESHORT:
            raise RuntimeError("STOI input shorter than one 256-sample frame at 10 kHz")
        _native.check(rc, "STOI")
        return s, e

    def _finish(self, stois: torch.Tensor, estois: torch.Tensor) -> list[dict[str, float]]:
        t = torch.stack([stois.float(), estois.float()])
        if t.is_cuda:  # the dicts are built while the GPU computes, then filled
            res, host = _native.list_from_device(self, t, ("STOI", "ESTOI"))
            nan_all = bool(np.isnan(host[0]).all())
        else:
            res, nan_all = None, bool(torch.isnan(t[0]).all())
        if nan_all:  # no utterance has a 30-frame segment (STOI.py:162-165)
            warnings.warn("Not enough non-silent frames. Please check your sound files", RuntimeWarning, stacklevel=3)
            raise TypeError("iteration over a 0-d tensor")
        return res if res is not None else _native.score_list(t, ("STOI", "ESTOI"))

    def _resample_cpu(self, x: torch.Tensor, sr: int) -> torch.Tensor:
        if sr == self.sample_rate:
            return self.resampler(x)
        from .resample import Resample
        return Resample(sr, self.EXPECTED_SAMPLING_RATE)(x)

    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths=None) -> list[dict[str, float]]:
        assert clean_speech is not None
        with torch.no_grad():
            return self._finish(*self.scores(clean_speech, denoised_speech, self.EXPECTED_SAMPLING_RATE,
                                             lengths=lengths))

    def __call__(self, clean_speech, denoised_speech, lengths=None) -> list[dict[str, float]]:
        if self.device == "cuda" and clean_speech is not None:
            # GPU: resampling is fused into the STOI kernels -- skip BaseMetric's resampler
            clean_speech, denoised_speech, lengths = self.split_ragged(clean_speech, denoised_speech, lengths)
            if clean_speech.shape != denoised_speech.shape:
                raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
            clean = torch.atleast_2d(clean_speech)
            noisy = torch.atleast_2d(denoised_speech)
            if not self.fans_out():  # (a multi-device metric's shards copy their own rows)
                clean, noisy = clean.to(self.home_device()), noisy.to(self.home_device())
            with torch.no_grad():
                return self._finish(*self.scores(clean, noisy, self.sample_rate, lengths=lengths))
        return super().__call__(clean_speech, denoised_speech, lengths)
