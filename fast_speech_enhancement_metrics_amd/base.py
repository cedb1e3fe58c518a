"""BaseMetric -- the reference's drop-in boundary (fast_se_metrics/base.py:6-43), unchanged API.

``metric = PESQ(sample_rate, use_gpu)`` then ``metric(clean, denoised) -> list[dict]``.
``use_gpu=True`` runs the gfx950 HIP engine (libfsem); it raises at construction if the
engine is missing -- there is no silent fallback.  ``use_gpu=False`` runs the package's
own CPU implementation (``_cpu.py``), the reference's CPU mode.
"""
from __future__ import annotations

import functools
from abc import ABC, abstractmethod

import torch

from . import _native
from .batching import as_lengths, pad_batch, resampled_lengths
from .resample import Resample


class BaseMetric(ABC):
    higher_is_better: bool
    EXPECTED_SAMPLING_RATE: int

    def __init__(self, sample_rate: int = 16000, use_gpu: bool = False, *, devices=None):
        """``devices`` (extension; GPU only): None = the current device, as the reference; ``"all"``,
        a count, or a list of devices (repeats allowed) = each call's rows split over those
        devices from this one process (multidevice.py), scores returned on the first."""
        self.sample_rate = sample_rate
        self.device = "cuda" if use_gpu else "cpu"
        self.resampler = Resample(sample_rate, self.EXPECTED_SAMPLING_RATE)
        self.resampler.to(self.device)
        self.devices = None
        self._fanout = None
        if use_gpu:
            if not torch.cuda.is_available():
                raise RuntimeError("use_gpu=True but no HIP device is visible")
            _native.load()
            from .multidevice import FanOut, resolve_devices
            self.devices = resolve_devices(devices)
            if self.devices is not None:  # (one listed device: its own thread and stream alike)
                self._fanout = FanOut(self.devices)

    # ---- what a GPU metric keeps between calls (the drop-in call's pinned score buffers and
    # event per host thread and device, the last result list's fill handle, the fan-out's
    # threads and streams) is process state: it is dropped when a metric is copied or pickled
    # (the reference's BaseMetric is a plain object; copies of it stay possible) and rebuilt on use.
    _TRANSIENT = ("_fsem_tls", "_held_list", "_fanout")

    def release(self) -> None:
        """Free the pinned score buffers and the last result list this metric keeps for its next
        call (they are rebuilt on the next call)."""
        _native.release(self)

    def __getstate__(self):
        state = self.__dict__.copy()
        for k in self._TRANSIENT:
            state.pop(k, None)
        return state

    def __setstate__(self, state):
        self.__dict__.update(state)
        self._fanout = None
        if self.devices is not None:
            from .multidevice import FanOut
            self._fanout = FanOut(self.devices)

    def home_device(self):
        """Where results live: the first listed device of a multi-device metric, else ``.device``."""
        return self.device if self.devices is None else self.devices[0]

    def fan_out(self, score, clean, noisy, lengths, ncols: int, balance=None):
        """``score(clean_rows, noisy_rows, lengths_rows)`` over this metric's devices (multidevice.py)
        -> ncols [B] float32 tensors on the first listed device."""
        return self._fanout.run(score, torch.atleast_2d(clean), torch.atleast_2d(noisy), lengths, ncols,
                                balance_lengths=balance)

    def fans_out(self) -> bool:
        """This call's rows go to several devices (a multi-device metric, not already on a shard)."""
        if self._fanout is None:
            return False
        from .multidevice import in_shard
        return not in_shard()

    def prepare_audio(self, audio: torch.Tensor, lengths: torch.Tensor | None = None) -> torch.Tensor:
        """The reference's prepare_audio (base.py:16-21); with ``lengths`` each row is resampled as
        its unpadded self (Resample.forward).  A multi-device metric leaves rows at the expected
        rate where they are: each shard copies its own rows to its device."""
        audio = torch.atleast_2d(audio)
        if self.fans_out() and self.sample_rate == self.EXPECTED_SAMPLING_RATE:
            return audio
        home = self.home_device()
        audio = audio.to(home)
        if self.sample_rate != self.EXPECTED_SAMPLING_RATE:
            if self.devices is not None:
                # the engine launches on the current HIP device (include/fsem.h): make the home
                # device current while its stream resamples (devices=[1, ...] called with 0 current)
                with torch.cuda.device(home):
                    audio = self.resampler(audio, lengths)
            else:
                audio = self.resampler(audio, lengths)
        return audio

    def prepare_inputs(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths: torch.Tensor | None = None):
        if clean_speech is not None and clean_speech.shape != denoised_speech.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        if clean_speech is not None:
            clean_speech = self.prepare_audio(clean_speech, lengths)
        denoised_speech = self.prepare_audio(denoised_speech, lengths)
        return clean_speech, denoised_speech

    @abstractmethod
    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths: torch.Tensor | None = None) -> list[dict[str, float]]:
        raise NotImplementedError

    def __call__(self, clean_speech, denoised_speech, lengths=None) -> list[dict[str, float]]:
        """The reference's call (base.py:41-43), extended to ragged batches: lists of 1-D
        utterances, or padded [B, L] tensors with per-row ``lengths`` (see batching.py)."""
        clean_speech, denoised_speech, lengths = self.split_ragged(clean_speech, denoised_speech, lengths)
        # with lengths, the resampler sees each row as the row alone would be (zeros past it)
        clean_speech, denoised_speech = self.prepare_inputs(clean_speech, denoised_speech, lengths)
        if lengths is None:
            return self.compute_metric(clean_speech, denoised_speech)
        lengths = resampled_lengths(lengths, self.sample_rate, self.EXPECTED_SAMPLING_RATE)
        return self.compute_metric(clean_speech, denoised_speech, lengths=lengths)

    @staticmethod
    def split_ragged(clean_speech, denoised_speech, lengths):
        """-> (clean, denoised, lengths | None) with lengths validated against the row capacity."""
        if isinstance(denoised_speech, (list, tuple)):
            if lengths is not None:
                raise ValueError("pass either lists of utterances or padded tensors with lengths")
            return pad_batch(clean_speech, denoised_speech)
        if lengths is not None:
            d = torch.atleast_2d(denoised_speech)
            lengths = as_lengths(lengths, d.shape[0], d.shape[-1])
        return clean_speech, denoised_speech, lengths


def zero_tail(x: torch.Tensor | None, lengths: torch.Tensor) -> torch.Tensor | None:
    """Zero every sample of row b at or past lengths[b]."""
    if x is None:
        return None
    x = torch.atleast_2d(x)
    t = torch.arange(x.shape[-1], device=x.device)
    return torch.where(t[None, :] < lengths.to(x.device, torch.int64)[:, None], x, torch.zeros((), dtype=x.dtype,
                                                                                               device=x.device))


def device_lengths(lengths, batch: int, capacity: int, device) -> torch.Tensor:
    """Validated int32 per-row lengths on `device` (the C-ABI's `lengths` array)."""
    if isinstance(lengths, torch.Tensor) and lengths.is_cuda and lengths.dtype == torch.int32 \
            and lengths.numel() == batch and lengths.device == torch.device(device):
        # trusted device array on the rows' device: no host round trip (the kernels clamp each
        # length to [0, L])
        return lengths.contiguous()
    return as_lengths(lengths, batch, capacity).to(device)


def same_device(clean: torch.Tensor, noisy: torch.Tensor) -> None:
    """The engine reads both operands on one device, as torch's own ops in the reference require
    (a host pointer handed to a kernel would fault the GPU instead of raising)."""
    if clean.device != noisy.device:
        raise RuntimeError("Expected all tensors to be on the same device, but found at least two devices, "
                           f"{clean.device} and {noisy.device}!")


def as_rows(x: torch.Tensor) -> torch.Tensor:
    """float32 [B, L] with unit stride along time (row stride = x.stride(0))."""
    x = torch.atleast_2d(x)
    if x.dtype != torch.float32:
        x = x.to(torch.float32)
    if x.dim() != 2 or x.stride(-1) != 1 or x.stride(0) < x.shape[1]:
        x = x.reshape(-1, x.shape[-1]).contiguous()
    return x


def noisy_shape(x) -> tuple:
    return tuple(torch.atleast_2d(torch.as_tensor(x)).shape) if x is not None else ()


def check_row_rate(metric, sample_rate: int | None) -> int:
    """Rate of the rows handed to ``metric.scores``.  None means the metric's expected rate, which
    is only unambiguous when the metric was constructed for that rate: a metric built for another
    rate must be told (otherwise its rows would silently be scored at the wrong rate)."""
    if sample_rate is None:
        if metric.sample_rate != metric.EXPECTED_SAMPLING_RATE:
            raise ValueError(f"{type(metric).__name__}({metric.sample_rate}).scores: pass sample_rate= (the rate of "
                             f"the rows; {metric.EXPECTED_SAMPLING_RATE} if they are already resampled)")
        return int(metric.EXPECTED_SAMPLING_RATE)
    return int(sample_rate)


@functools.lru_cache(maxsize=32)
def _resampler(orig: int, new: int) -> Resample:
    # one module per rate pair, kept on the host: its CUDA path runs in libfsem and never reads the
    # kernel buffer, so no per-call host -> device copy (which would wait for the stream to drain)
    return Resample(orig, new)


def resample_rows(clean, noisy, lengths, orig: int, new: int):
    """(clean, noisy, lengths) resampled orig -> new, each row as the row alone when ``lengths`` is
    given (BaseMetric.prepare_audio, base.py:19-20); lengths become the resampled lengths."""
    rs = _resampler(int(orig), int(new))
    noisy = torch.atleast_2d(noisy)
    lens = None
    if lengths is not None:
        lens = device_lengths(lengths, noisy.shape[0], noisy.shape[-1], noisy.device)
    clean = rs(torch.atleast_2d(clean), lens) if clean is not None else None
    noisy = rs(noisy, lens)
    if lens is not None:
        lens = resampled_lengths(lens, orig, new).to(noisy.device)
    return clean, noisy, lens
