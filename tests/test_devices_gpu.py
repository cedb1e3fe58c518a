"""Operands on two devices (a GPU row and a host row, or host-held per-row lengths) at the engine
entries: refused before any launch with torch's own message (the reference's torch ops refuse the
mix as well) -- a host pointer handed to a kernel would fault the GPU; the drop-in call moves both
rows to the metric's device first, as BaseMetric.prepare_audio does (base.py:19-20)."""
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
from fast_speech_enhancement_metrics_amd.alignment import time_align, time_align_segments

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rows():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    g = torch.Generator().manual_seed(3)
    c = torch.randn(2, 32000, generator=g) * 0.1
    n = c + 0.05 * torch.randn(2, 32000, generator=g)
    return c, n


def test_mixed_devices_refused(rows):
    c, n = rows
    cg = c.cuda()
    calls = [lambda: PESQ(16000, use_gpu=True).scores(cg, n), lambda: STOI(16000, use_gpu=True).scores(cg, n, 16000),
             lambda: PESQ_STOI(16000, use_gpu=True).scores(cg, n), lambda: time_align(cg, n),
             lambda: time_align_segments(cg, n, mode="p862")]
    for call in calls:
        with pytest.raises(RuntimeError, match="same device"):
            call()


def test_dropin_call_moves_host_rows(rows):
    c, n = rows
    m = PESQ_STOI(16000, use_gpu=True)
    want = m(c.cuda(), n.cuda())
    assert m(c, n.cuda()) == want and m(c, n) == want


def test_host_lengths_with_device_rows(rows):
    c, n = rows
    m = PESQ_STOI(16000, use_gpu=True)
    lens = torch.tensor([32000, 20000], dtype=torch.int32)
    a = [t.cpu() for t in m.scores(c.cuda(), n.cuda(), lengths=lens)]
    b = [t.cpu() for t in m.scores(c.cuda(), n.cuda(), lengths=lens.cuda())]
    for x, y in zip(a, b):
        assert torch.equal(x, y)
