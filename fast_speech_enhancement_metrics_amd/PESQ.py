"""PESQ-wb metric -- drop-in for the reference's ``fast_se_metrics.PESQ`` (PESQ.py:13-245).

P.862-like wideband model without time alignment and with IIR level alignment
(reference PESQ.py:17-23).  ``use_gpu=True``: the whole per-utterance pipeline runs in
libfsem's gfx950 kernels (``fsem_pesq_wb_f32``) with one device->host copy of the scores;
``use_gpu=False``: the package's CPU implementation.
"""
from __future__ import annotations

import torch

from . import _cpu, _native
from .bark import BarkFilterBank
from .base import BaseMetric, as_rows, check_row_rate, device_lengths, noisy_shape, resample_rows, same_device
from .loudness import Loudness
from .spectrogram import Spectrogram


def _unit_rows(x: torch.Tensor, lengths=None) -> torch.Tensor:
    """Rows scaled by a power of two (exact) to a peak in [1, 2) of their first lengths[b] samples;
    zero / non-finite rows as they are."""
    a = x
    if lengths is not None:
        t = torch.arange(x.shape[1], device=x.device)
        a = x.masked_fill(t[None, :] >= torch.as_tensor(lengths, device=x.device).reshape(-1, 1), 0.0)
    peak = torch.linalg.vector_norm(a, ord=float("inf"), dim=1)  # max |x|: one pass over the rows
    ex = torch.where((peak > 0) & torch.isfinite(peak), torch.floor(torch.log2(peak)), torch.zeros_like(peak))
    return x * torch.exp2(-ex).to(x.dtype)[:, None]  # a power of two: exact, as ldexp


def _wb_frames(lib, clean: torch.Tensor, noisy: torch.Tensor, lens):
    """(distances [2, B], per-frame disturbances [B, 2, F]) of 16 kHz rows on the GPU through the
    whole-metric entry (fsem_pesq_wb_frames_f32: its range handling, no host-side row scaling)."""
    clean = as_rows(clean)
    noisy = as_rows(noisy)
    B, L = clean.shape
    F = lib.fsem_pesq_frames(L)
    if F < 20 and lens is None:
        raise RuntimeError(f"maximum size for tensor at dimension 1 is {max(F, 0)} but size is 20")
    if clean.stride(0) != noisy.stride(0) or L % 4 or not (clean.is_contiguous() and noisy.is_contiguous()):
        pad = (-L) % 4
        clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
        noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
    mos = torch.empty(B, dtype=torch.float32, device=clean.device)
    dist = torch.empty(2, B, dtype=torch.float32, device=clean.device)
    frames = torch.full((B, 2, F), float("nan"), device=clean.device)
    ws = _native.workspace(lib.fsem_pesq_workspace_bytes(B, L), clean.device)
    _native.check(lib.fsem_pesq_wb_frames_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                                              lens.data_ptr() if lens is not None else None, mos.data_ptr(),
                                              dist.data_ptr(), frames.data_ptr(), ws.data_ptr(), ws.numel(),
                                              _native.stream_handle(clean.device)), "PESQ frames")
    return dist[0], frames


class PESQ(BaseMetric):
    higher_is_better = True
    EXPECTED_SAMPLING_RATE = 16000

    def __init__(self, sample_rate: int = 16000, use_gpu: bool = False, *, time_align=False,
                 max_delay: int = 16000, devices=None):
        """``time_align`` (extension, off by default as in the reference, PESQ.py:19-22): shift each
        degraded row by its estimated delay before scoring (``alignment.time_align``, P.862-style;
        ``max_delay`` samples at 16 kHz bounds the search): True or "row" -- one delay per row;
        "utterance" -- P.862's per-utterance delays, the row realigned segment by segment;
        "p862" -- the same with P.862's histogram fine stage and recursive utterance split.  The
        delays of the last scored batch (per row; in the segment modes each row's longest
        segment's) are kept in ``last_delays``.  ``devices``: see BaseMetric (multi-device calls)."""
        super().__init__(sample_rate, use_gpu, devices=devices)
        if time_align not in (False, True, "row", "utterance", "p862"):
            raise ValueError('time_align must be False, True, "row", "utterance" or "p862"')
        self.time_align = "row" if time_align is True else time_align
        self.max_delay = int(max_delay)
        self.last_delays = None

    @staticmethod
    def equalize_ranges(clean_speech: torch.Tensor, noisy_speech: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
        """Both rows divided by their joint peak |x| (PESQ.py:115-121).  The engine skips this step:
        it cancels under the level alignment (amplitude range)."""
        m = torch.maximum(clean_speech.abs().amax(dim=1, keepdim=True), noisy_speech.abs().amax(dim=1, keepdim=True))
        return clean_speech / m, noisy_speech / m

    # ------------------------------------------------------------------ reference attributes
    # The reference's constructor attributes (PESQ.py:63-90), on the metric's device, built on
    # first access (the engine carries its own copies in constant memory).
    @property
    def power_filter(self) -> torch.Tensor:
        """[2, 11] (b; a) of the order-5 Butterworth band-pass 325-3250 Hz at 16 kHz (PESQ.py:80-81)."""
        if getattr(self, "_power_filter", None) is None:
            import numpy as np
            from scipy.signal import butter
            out = np.asarray(butter(5, [325, 3250], fs=16000, btype="band"))
            self._power_filter = torch.as_tensor(out, device=self.device, dtype=torch.float32)
        return self._power_filter

    @property
    def pre_filter(self) -> torch.Tensor:
        """[2, 3] (b; a) of the pre-emphasis IIR (PESQ.py:84-88)."""
        if getattr(self, "_pre_filter", None) is None:
            self._pre_filter = torch.tensor([[2.740826, -5.4816519, 2.740826], [1.0, -1.9444777, 0.94597794]],
                                            device=self.device, dtype=torch.float32)
        return self._pre_filter

    @property
    def taper_weights(self) -> torch.Tensor:
        """[15] edge taper (k + 1) / 16 of the first / last 15 samples (PESQ.py:90)."""
        if getattr(self, "_taper_weights", None) is None:
            self._taper_weights = torch.linspace(0, 15, 16, device=self.device)[1:] / 16.0
        return self._taper_weights

    @property
    def to_spec(self) -> Spectrogram:
        """Hann-512 / hop-256 power spectrogram, center=False (PESQ.py:63-71)."""
        if getattr(self, "_to_spec", None) is None:
            self._to_spec = Spectrogram(win_length=512, n_fft=512, hop_length=256, window_fn=torch.hann_window,
                                        power=2, normalized=False, center=False).to(self.device)
        return self._to_spec

    @property
    def filter_bank(self) -> BarkFilterBank:
        """P.862 Bark filterbank, 256 bins -> 49 bands (PESQ.py:74)."""
        if getattr(self, "_filter_bank", None) is None:
            self._filter_bank = BarkFilterBank(256, 49, device=self.device)
        return self._filter_bank

    @property
    def loudness(self) -> Loudness:
        """Zwicker loudness model over the 49 bands (PESQ.py:77)."""
        if getattr(self, "_loudness", None) is None:
            self._loudness = Loudness(49, device=self.device)
        return self._loudness

    # ------------------------------------------------------------------ stage methods
    # The reference's pipeline stages (PESQ.py:92-230) on [rows, samples] tensors of 16 kHz
    # speech.  On the GPU the band-pass power and the Bark bands come from the engine's front end
    # (fsem_pesq_front_f32) and the disturbances from its back end (fsem_pesq_distances_f32); the
    # remaining stages are short torch expressions on the metric's device.  Scores do not go
    # through these methods: compute_metric runs the whole engine in one call.
    def _front(self, speech: torch.Tensor):
        """Engine front end on any number of rows -> (unscaled Bark bands [N, F, 49], sum of the
        squared band-pass output [N]), float64.  Rows go in scaled by a power of two to a peak
        in [1, 2) (exact) and the results come back at the rows' own scale in float64, so the
        float32 stage outputs cannot overflow for any finite input."""
        x = as_rows(speech)
        N, L = x.shape
        peak = x.abs().amax(dim=1)
        ex = torch.where((peak > 0) & torch.isfinite(peak), torch.floor(torch.log2(peak)), torch.zeros_like(peak))
        x = _unit_rows(x).contiguous()
        if L % 4 or N % 2:
            x = torch.nn.functional.pad(x, (0, (-L) % 4))
            if N % 2:
                x = torch.cat([x, x[-1:]], 0)  # the front end takes rows in (ref, deg) halves
            x = x.contiguous()
        h = x.shape[0] // 2
        lib = _native.load()
        F = lib.fsem_pesq_frames(L)
        if F < 1:
            raise RuntimeError("PESQ input shorter than one 512-sample frame")
        fld = (F + 31) // 32 * 32
        bark = torch.empty(2 * h, 49, fld, device=x.device)
        power = torch.empty(2 * h, device=x.device)
        ws = _native.workspace(lib.fsem_pesq_front_workspace_bytes(h, L), x.device)
        _native.check(lib.fsem_pesq_front_f32(x[:h].data_ptr(), x[h:].data_ptr(), h, L, x.stride(0), None,
                                              bark.data_ptr(), power.data_ptr(), ws.data_ptr(), ws.numel(),
                                              _native.stream_handle(x.device)), "PESQ front")
        g = torch.exp2(2 * ex.double())
        return bark[:N, :, :F].transpose(1, 2).double() * g[:, None, None], power[:N].double() * g

    def align_level(self, speech: torch.Tensor) -> torch.Tensor:
        """Rows scaled to band-pass power 1e7 (PESQ.py:92-102): x * sqrt(1e7 / P) with
        P = sum(bandpass(x)^2) / (L + 5120) / 1.04684."""
        speech = torch.atleast_2d(speech)
        L = speech.shape[1]
        if speech.is_cuda and _cpu.pesq_frames(L) >= 1:
            p = self._front(speech)[1]
        else:
            # host float64 cascade: CPU rows, and rows shorter than one 512-sample frame (the
            # engine's front end frames what it filters; the reference filters any length)
            p = torch.from_numpy(_cpu.bandpass_power(speech.detach().to("cpu", torch.float64).numpy()))
        gain = _cpu.level_scale(p, L).sqrt().to(speech.device, speech.dtype)
        return speech * gain[:, None]

    def pre_emphasize(self, speech: torch.Tensor) -> torch.Tensor:
        """Edge taper (in place on ``speech``, as the reference) and the pre-emphasis IIR
        (PESQ.py:104-113); float32 rows stay float32, on the GPU the filter runs on the device
        (fsem_pre_emphasize_f32, torchaudio's float32 evaluation order)."""
        w = self.taper_weights.to(speech.device, speech.dtype)
        speech[:, :15] *= w
        speech[:, -15:] *= torch.flip(w, dims=(0,))
        if speech.is_cuda:
            x = as_rows(speech)
            y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
            lib = _native.load()
            _native.check(lib.fsem_pre_emphasize_f32(x.data_ptr(), x.shape[0], x.shape[1], x.stride(0), y.data_ptr(),
                                                     y.stride(0), _native.stream_handle(x.device)), "pre-emphasis")
            return y.to(speech.dtype)
        from scipy.signal import lfilter
        y = lfilter(_cpu._PRE_B, _cpu._PRE_A, speech.detach().to("cpu", torch.float64).numpy(), axis=1)
        return torch.from_numpy(y).to(speech.device, speech.dtype)

    def get_bark_bands(self, speech: torch.Tensor) -> torch.Tensor:
        """[N, L] rows -> [N, F, 49] float64 Bark power bands after level alignment and
        pre-emphasis (PESQ.py:123-140)."""
        speech = torch.atleast_2d(speech)
        if not speech.is_cuda:
            return _cpu.bark_of_rows(speech).to(speech.device)
        bark, p = self._front(speech)
        return bark * _cpu.level_scale(p, speech.shape[1])[:, None, None]

    def equalize_bark_bands(self, clean_bark_bands: torch.Tensor, noisy_bark_bands: torch.Tensor):
        """(clean, noisy) Bark bands after the band and frame power equalisation (PESQ.py:142-166)."""
        return _cpu.equalize(clean_bark_bands, noisy_bark_bands)

    def get_overlapping_sums(self, disturbance: torch.Tensor) -> torch.Tensor:
        """[B, F] -> [B]: L6 over 20-frame windows (hop 10), then L2 over windows (PESQ.py:168-172)."""
        return _cpu.overlapping_sums(disturbance)

    def get_disturbances(self, clean_speech: torch.Tensor, noisy_speech: torch.Tensor):
        """(symmetric, asymmetric) distances [B] of 16 kHz pairs (PESQ.py:174-230); MOS =
        0.999 + 4 / (1 + exp(-1.3669 (4.5 - 0.1 sym - 0.0309 asym) + 3.8224))."""
        clean = as_rows(clean_speech)
        noisy = as_rows(noisy_speech)
        if clean.shape != noisy.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        if not clean.is_cuda:
            return _cpu.pesq_distances(clean, noisy)
        sym, asym, _ = self.frame_disturbances(clean, noisy)
        return sym, asym

    def frame_disturbances(self, clean_speech: torch.Tensor, noisy_speech: torch.Tensor, lengths=None):
        """Engine back-end intermediates of 16 kHz pairs: (symmetric distance [B], asymmetric
        distance [B], per-frame disturbances [B, 2, F] -- symmetric then asymmetric, after the
        frame weighting and the clamp at 45, PESQ.py:222-224).  GPU only (the stage entry
        fsem_pesq_distances_f32); rows under 20 frames give NaN distances."""
        # each signal is level-aligned on its own (PESQ.py:92-102), so scaling a row by a power of
        # two changes nothing but the range: rows go in with peaks in [1, 2), as _front
        same_device(as_rows(clean_speech), as_rows(noisy_speech))
        clean = _unit_rows(as_rows(clean_speech), lengths)
        noisy = _unit_rows(as_rows(noisy_speech), lengths)
        lib = _native.load()
        B, L = clean.shape
        F = lib.fsem_pesq_frames(L)
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if F < 20 and lens is None:
            raise RuntimeError(f"maximum size for tensor at dimension 1 is {max(F, 0)} but size is 20")
        if clean.stride(0) != noisy.stride(0) or L % 4:
            pad = (-L) % 4
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        fld = (F + 31) // 32 * 32
        bark = torch.empty(2 * B, 49, fld, device=clean.device)
        power = torch.empty(2 * B, device=clean.device)
        st = _native.stream_handle(clean.device)
        ws = _native.workspace(max(lib.fsem_pesq_front_workspace_bytes(B, L),
                                   lib.fsem_pesq_distances_workspace_bytes(B, L)), clean.device)
        lp = lens.data_ptr() if lens is not None else None
        _native.check(lib.fsem_pesq_front_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0), lp,
                                              bark.data_ptr(), power.data_ptr(), ws.data_ptr(), ws.numel(), st),
                      "PESQ front")
        dist = torch.empty(2, B, device=clean.device)
        frames = torch.full((B, 2, F), float("nan"), device=clean.device)
        _native.check(lib.fsem_pesq_distances_f32(bark.data_ptr(), power.data_ptr(), B, L, lp, dist.data_ptr(),
                                                  frames.data_ptr(), ws.data_ptr(), ws.numel(), st),
                      "PESQ distances")
        return dist[0], dist[1], frames

    # ------------------------------------------------------------------ device paths
    def scores(self, clean_speech: torch.Tensor, denoised_speech: torch.Tensor, lengths=None,
               sample_rate: int | None = None) -> torch.Tensor:
        """Per-utterance MOS as a tensor on the metric's device (no host sync on GPU).

        Rows at ``sample_rate``; None means rows already at 16 kHz, which requires a 16 kHz metric
        (a ``PESQ(8000)`` must be told its rows' rate, or it would score them as 16 kHz).  Other
        rates are resampled to 16 kHz first, each row as the row alone (BaseMetric.prepare_audio,
        base.py:19-20).  ``lengths`` (optional, [B] ints at that rate): row b holds lengths[b]
        samples and scores as the reference would on that unpadded row alone; rows under 20
        frames give NaN.
        """
        sr = check_row_rate(self, sample_rate)
        if noisy_shape(clean_speech) != noisy_shape(denoised_speech):
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        aligned = getattr(self, "time_align", False)
        if self.fans_out():
            def shard(c, n, lk):
                mos, delays = self._rows_scores(c, n, lk, sr)
                return (mos, delays.to(torch.int32)) if aligned else mos  # FanOut keeps the dtype: exact delays

            cols = self.fan_out(shard, clean_speech, denoised_speech, lengths, 2 if aligned else 1, balance=lengths)
            if aligned:
                self.last_delays = cols[1].to(torch.int32)
            return cols[0]
        mos, delays = self._rows_scores(clean_speech, denoised_speech, lengths, sr)
        if aligned:
            self.last_delays = delays
        return mos

    def _rows_scores(self, clean_speech, denoised_speech, lengths, sr: int):
        """(mos [B], delays [B] or None) of rows at rate ``sr`` on their own device (one engine call)."""
        delays = None
        if sr != self.EXPECTED_SAMPLING_RATE:
            clean_speech, denoised_speech, lengths = resample_rows(clean_speech, denoised_speech, lengths, sr,
                                                                   self.EXPECTED_SAMPLING_RATE)
        clean = as_rows(clean_speech)
        noisy = as_rows(denoised_speech)
        B, L = clean.shape
        if noisy.shape != clean.shape:
            raise Exception("`clean_speech` and `denoised_speech` should have the same shape.")
        same_device(clean, noisy)
        if getattr(self, "time_align", False) == "p862":
            mos, delays, _, _ = self.p862_scores(clean, noisy, lengths)
            return mos, delays
        if getattr(self, "time_align", False):
            from .alignment import time_align
            noisy, delays = time_align(clean, noisy, lengths, self.max_delay, mode=self.time_align)
        lib = _native.load() if clean.is_cuda else None
        if lib is None:
            if lengths is None:
                return _cpu.rows_parallel(_cpu.pesq, clean, noisy), delays
            return _cpu.per_row(_cpu.pesq, clean, noisy, device_lengths(lengths, B, L, "cpu")), delays
        F = lib.fsem_pesq_frames(L)
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        if F < 20 and lens is None:
            # the reference's unfold(1, size=20, step=10) fails here (PESQ.py:169)
            raise RuntimeError(f"maximum size for tensor at dimension 1 is {max(F, 0)} but size is 20")
        if clean.stride(0) != noisy.stride(0) or L % 4:
            # rows must be readable up to ceil4(L) floats (include/fsem.h): pad odd lengths
            pad = (-L) % 4
            clean = torch.nn.functional.pad(clean, (0, pad)).contiguous()
            noisy = torch.nn.functional.pad(noisy, (0, pad)).contiguous()
        mos = torch.empty(B, dtype=torch.float32, device=clean.device)
        ws = _native.workspace(lib.fsem_pesq_workspace_bytes(B, L), clean.device)
        _native.check(lib.fsem_pesq_wb_f32(clean.data_ptr(), noisy.data_ptr(), B, L, clean.stride(0),
                                           lens.data_ptr() if lens is not None else None,
                                           mos.data_ptr(), ws.data_ptr(), ws.numel(),
                                           _native.stream_handle(clean.device)), "PESQ")
        return mos, delays

    def p862_scores(self, clean_speech: torch.Tensor, noisy_speech: torch.Tensor, lengths=None):
        """The ``time_align="p862"`` scores of 16 kHz rows (extension, not in the reference,
        PESQ.py:19-22): the P.862-mode alignment (``alignment.time_align_segments``), the aligned
        rows' per-frame disturbances, P.862's realignment of bad intervals
        (``alignment.realign_bad_intervals``), the realigned rows' disturbances (only rows with an
        interval), and the MOS of the frames each interval scores better with
        (``fsem_pesq_pool_f32``).  Returns (mos [B] float32, delays [B], n_bad [B], bad [B, 16, 3])
        on the rows' device (CPU rows: _cpu.pesq_p862, mos float64)."""
        from . import alignment
        clean = as_rows(clean_speech)
        noisy = as_rows(noisy_speech)
        same_device(clean, noisy)
        B, L = clean.shape
        max_delay = getattr(self, "max_delay", alignment.DEFAULT_MAX_DELAY)
        if not clean.is_cuda:
            lens = None if lengths is None else device_lengths(lengths, B, L, "cpu")
            return _cpu.pesq_p862(clean, noisy, lens, max_delay)
        lib = _native.load()
        lens = device_lengths(lengths, B, L, clean.device) if lengths is not None else None
        aligned, delays, nseg, starts, sdel = alignment.time_align_segments(clean, noisy, lens, max_delay, mode="p862")
        ds, fr1 = _wb_frames(lib, clean, aligned, lens)
        n_bad, bad, second = alignment.realign_bad_intervals(clean, noisy, aligned, fr1, nseg, starts, sdel, lens)
        fr2 = fr1
        rows = torch.nonzero(n_bad).flatten()  # host sync: the second scoring covers these rows only
        if 2 * rows.numel() > B:
            # most rows: score the whole batch again rather than gather them (a row without an
            # interval has second == aligned, so its frames come out as fr1's)
            _, fr2 = _wb_frames(lib, clean, second, lens)
        elif rows.numel():
            fr2 = fr1.clone()
            _, sub = _wb_frames(lib, clean[rows], second[rows], None if lens is None else lens[rows])
            fr2[rows] = sub
        mos = torch.empty(B, dtype=torch.float32, device=clean.device)
        _native.check(lib.fsem_pesq_pool_f32(fr1.data_ptr(), fr2.data_ptr(), ds.data_ptr(), B, L,
                                             lens.data_ptr() if lens is not None else None, n_bad.data_ptr(),
                                             bad.data_ptr(), mos.data_ptr(), _native.stream_handle(clean.device)),
                      "PESQ pool")
        return mos, delays, n_bad, bad

    def compute_metric(self, clean_speech: torch.Tensor | None, denoised_speech: torch.Tensor,
                       lengths=None) -> list[dict[str, float]]:
        assert clean_speech is not None
        with torch.inference_mode():
            mos = self.scores(clean_speech, denoised_speech, lengths, sample_rate=self.EXPECTED_SAMPLING_RATE)
            if not mos.is_cuda:
                return _native.score_list(mos.reshape(1, -1), ("PESQ",))
            return _native.list_from_device(self, mos.reshape(1, -1), ("PESQ",))[0]
