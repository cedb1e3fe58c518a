"""ORACLE / TEST INFRASTRUCTURE ONLY -- stand-in for torchaudio 2.8.0 (absent from the image).

Put ``oracle/ta_shim`` first on ``sys.path`` ONLY inside ``tests/golden/make_golden.py`` so
that the reference's own ``fast_se_metrics`` package can be imported and run on the CPU
to produce golden vectors.  Each operator restates torchaudio's published algorithm
using the same torch primitives torchaudio itself calls (``conv1d``, ``torch.stft``),
plus the C restatement of torchaudio's sequential lfilter loop.
"""
from . import functional, transforms  # noqa: F401

__version__ = "2.8.0-oracle-restatement"
