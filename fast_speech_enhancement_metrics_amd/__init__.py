"""MI355X-native batched PESQ-wb and STOI/ESTOI (drop-in for kcoost/fast_speech_enhancement_metrics).

    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    PESQ(sample_rate=16000, use_gpu=True)(clean, denoised)  -> [{"PESQ": ...}, ...]
    STOI(sample_rate=16000, use_gpu=True)(clean, denoised)  -> [{"STOI": ..., "ESTOI": ...}, ...]
    PESQ_STOI(16000, use_gpu=True)(clean, denoised)        -> [{"PESQ", "STOI", "ESTOI"}, ...]  (one pass)

Ragged batches: pass lists of 1-D utterances, or padded [B, L] tensors with ``lengths=``.
"""
from .base import BaseMetric
from .PESQ import PESQ
from .STOI import STOI
from .joint import PESQ_STOI
from .alignment import time_align

__all__ = ["BaseMetric", "PESQ", "STOI", "PESQ_STOI", "time_align"]
