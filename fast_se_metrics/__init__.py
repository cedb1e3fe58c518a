"""Drop-in import path of the reference package: ``from fast_se_metrics import PESQ, STOI``.

Only the hot-path metrics (PESQ-wb, STOI/ESTOI) are provided; SDR, LSD, DNSMOS and
SpeechBERTScore of the reference are out of scope.
"""
from fast_se_metrics.PESQ import PESQ  # noqa: F401  (module path first, then the class, as the reference)
from fast_se_metrics.STOI import STOI  # noqa: F401

__all__ = ["STOI", "PESQ"]
