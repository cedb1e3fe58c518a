"""Drop-in module path ``fast_se_metrics.STOI`` (reference fast_se_metrics/STOI.py)."""
from fast_speech_enhancement_metrics_amd.STOI import STOI  # noqa: F401

__all__ = ["STOI"]
