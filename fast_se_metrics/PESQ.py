"""Drop-in module path ``fast_se_metrics.PESQ`` (reference fast_se_metrics/PESQ.py)."""
from fast_speech_enhancement_metrics_amd.PESQ import PESQ  # noqa: F401

__all__ = ["PESQ"]
