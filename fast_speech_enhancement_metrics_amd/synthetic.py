"""Synthetic speech-like (clean, noisy) pairs for tests and benchmarks.

The reference's data (``benchmarking/dataloading.py``: HF ``MLCommons/peoples_speech`` speech
+ ``nccratliri/wing-flap-noise-audio-examples`` noise) is a network fetch that is not
available here, so this module synthesises signals of the same shape and statistics:

* voiced harmonic source, f0 90-250 Hz with slow vibrato, 3-formant spectral envelope;
* 3-6 Hz syllabic amplitude modulation and 0.3-1 s silent gaps (exercises PESQ's silent-frame
  logic and STOI's 40 dB voice-activity selection);
* amplitude-modulated broadband noise mixed at an SNR drawn uniformly from
  [snr_low, snr_high] dB with the reference's recipe (``dataloading.py:63-72``);
* both signals quantised to the int16 grid (x = k / 32768), so fixtures store them exactly.

Runs with torch on any device (the benchmark generates its batch directly in HBM).
"""
from __future__ import annotations

import math

import torch


def speech_like_pairs(batch: int, length: int, sample_rate: int = 16000, seed: int = 42,
                      device: str | torch.device = "cpu", snr_low: float = -5.0,
                      snr_high: float = 25.0, quantize: bool = True):
    """Return (clean [B, L] f32, noisy [B, L] f32, snr [B, 1] f32)."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))

    def rnd(*shape):
        return torch.rand(*shape, generator=g, device=dev, dtype=torch.float32)

    B, L = int(batch), int(length)
    t = torch.arange(L, device=dev, dtype=torch.float32) / sample_rate          # [L]
    f0b = 90.0 + 160.0 * rnd(B, 1)
    vib_rate = 0.3 + 1.2 * rnd(B, 1)
    vib_phase = 2 * math.pi * rnd(B, 1)
    f0 = f0b * (1.0 + 0.08 * torch.sin(2 * math.pi * vib_rate * t + vib_phase))  # [B, L]
    # instantaneous phase in cycles (float64 cumsum for long signals), wrapped to [0, 1)
    cyc = torch.cumsum(f0.double(), dim=1) / sample_rate
    cyc = (cyc - torch.floor(cyc)).float()
    del f0
    F1 = 300.0 + 600.0 * rnd(B, 1)
    F2 = 900.0 + 1600.0 * rnd(B, 1)
    F3 = 2300.0 + 1200.0 * rnd(B, 1)
    voiced = torch.zeros(B, L, device=dev)
    nyq = 0.45 * sample_rate
    for k in range(1, 33):
        fk = k * f0b                                                            # [B, 1]
        amp = (torch.exp(-0.5 * ((fk - F1) / 120.0) ** 2)
               + 0.7 * torch.exp(-0.5 * ((fk - F2) / 180.0) ** 2)
               + 0.4 * torch.exp(-0.5 * ((fk - F3) / 250.0) ** 2)
               + 0.05 / (1.0 + fk / 1000.0))
        amp = torch.where(fk < nyq, amp, torch.zeros_like(amp))
        ph = 2 * math.pi * ((k * cyc) - torch.floor(k * cyc))
        voiced += amp * torch.sin(ph)
    del cyc
    syl_rate = 3.0 + 3.0 * rnd(B, 1)
    syl = (0.5 + 0.5 * torch.sin(2 * math.pi * syl_rate * t + 2 * math.pi * rnd(B, 1))) ** 2
    gate_s = (torch.sin(2 * math.pi * (0.25 + 0.2 * rnd(B, 1)) * t + 2 * math.pi * rnd(B, 1))
              + 0.5 * torch.sin(2 * math.pi * (0.7 + 0.4 * rnd(B, 1)) * t + 2 * math.pi * rnd(B, 1)))
    gate = torch.clamp((gate_s + 0.6) * 6.0, 0.0, 1.0)
    clean = voiced * (0.15 + 0.85 * syl) * gate
    del voiced, syl, gate, gate_s
    clean = clean + 3e-4 * torch.randn(B, L, generator=g, device=dev)          # recording floor
    clean = clean / clean.abs().amax(dim=1, keepdim=True).clamp_min(1e-12) * (0.3 + 0.4 * rnd(B, 1))

    am = 1.0 + 0.6 * torch.sin(2 * math.pi * (8.0 + 20.0 * rnd(B, 1)) * t + 2 * math.pi * rnd(B, 1))
    noise = torch.randn(B, L, generator=g, device=dev) * am
    del am
    # reference mixing recipe (dataloading.py:63-72)
    speech_rms = clean.square().mean(dim=1, keepdim=True).sqrt()
    noise_rms = noise.square().mean(dim=1, keepdim=True).sqrt()
    snr = rnd(B, 1) * (snr_high - snr_low) + snr_low
    scale = speech_rms / (10 ** (snr / 20)) / (noise_rms + 1e-12)
    noisy = clean + scale * noise
    del noise
    if quantize:
        clean = torch.clamp(torch.round(clean * 32768.0), -32768, 32767) / 32768.0
        noisy = torch.clamp(torch.round(noisy * 32768.0), -32768, 32767) / 32768.0
    return clean.float().contiguous(), noisy.float().contiguous(), snr


def to_int16(x: torch.Tensor):
    """Exact int16 codes of an int16-grid float tensor."""
    return torch.round(x * 32768.0).to(torch.int16)


def from_int16(codes) -> torch.Tensor:
    return torch.as_tensor(codes).to(torch.float32) / 32768.0
