"""ORACLE -- TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's hot path (kcoost/fast_speech_enhancement_metrics,
``fast_se_metrics/PESQ.py``, ``STOI.py``, ``utils/bark.py``, ``utils/loudness.py``) and of
the torchaudio 2.8.0 operators it calls (``lfilter``, ``Resample``, ``Spectrogram``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this package, and only as the checker / the timed CPU baseline.  The product
package ``fast_speech_enhancement_metrics_amd`` never imports it.

Parity pinning: the restatement is checked against golden vectors produced by running
the reference's own ``PESQ``/``STOI`` classes in the build container
(``tests/golden/make_golden.py``); torchaudio is absent from the image, so those runs use
``oracle/ta_shim`` -- torch's own ``conv1d``/``stft`` (what torchaudio itself calls) plus the
C restatement of torchaudio's sequential lfilter loop (``oracle/c/lfilter_f32.c``).
"""
