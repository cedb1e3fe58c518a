"""The drop-in call's fast path (joint.py PESQ_STOI._fast_call: launch first, dicts built and the
previous call's list released while the GPU computes): the same list as the generic path,
bitwise; inputs it does not cover take the generic path; the reference's exceptions and warning
stay; the previous list's dicts are held until the next call and then released; the scores land
in the thread's mapped pinned buffer directly (no device copy), the same as through a copy."""
import gc
import sys
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pairs():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(12, 48000, 16000, seed=71, device="cuda")
    return c, n


def _generic(m, c, n):
    m._fast_ok = lambda *a: False  # instance override: the generic BaseMetric path
    try:
        return m(c, n)
    finally:
        del m._fast_ok


def test_fast_path_equals_generic_path(pairs):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    assert m._fast_ok(c, n)
    fast = m(c, n)
    slow = _generic(m, c, n)
    assert len(fast) == len(slow) == c.shape[0]
    for a, b in zip(fast, slow):
        assert list(a) == ["PESQ", "STOI", "ESTOI"]
        assert a == b and all(type(v) is float for v in a.values())
    # and the engine API's scores
    p, s, e = (t.cpu().numpy() for t in m.scores(c, n))
    np.testing.assert_array_equal(np.array([d["PESQ"] for d in fast], np.float32), p)
    np.testing.assert_array_equal(np.array([d["ESTOI"] for d in fast], np.float32), e)


def test_other_inputs_take_the_generic_path(pairs):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    want = m(c, n)
    assert not m._fast_ok(c[0], n[0])                       # 1-D
    assert not m._fast_ok(c.double(), n.double())           # dtype
    assert not m._fast_ok(c.cpu(), n.cpu())                 # host tensors
    assert not m._fast_ok(c[:, :-2], n[:, :-2])             # L % 4
    assert not m._fast_ok(c, n[:, :40000])                  # shape mismatch
    assert m(c.double(), n.double()) == want                # the reference's .to / dtype handling
    assert m(c.cpu(), n.cpu()) == want
    with pytest.raises(Exception, match="same shape"):
        m(c, n[:, :40000])


def test_short_input_raises_like_reference():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    m = PESQ_STOI(16000, use_gpu=True)
    x = torch.randn(2, 4000, device="cuda")
    assert m._fast_ok(x, x)
    with pytest.raises(RuntimeError):
        m(x, x)


def test_previous_list_is_held_until_next_call(pairs):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    r1 = m(c, n)
    d0 = r1[0]
    assert sys.getrefcount(d0) == 3  # the list's slot, d0, getrefcount's argument
    del r1
    gc.collect()
    assert sys.getrefcount(d0) == 3  # the list is still held by the metric (its fill handle)
    r2 = m(c, n)
    assert sys.getrefcount(d0) == 2  # released during the next call: d0 and the argument
    assert r2[0] == d0


def test_no_stoi_segment_warns_like_reference():
    """Rows long enough for PESQ (22 frames) but without a 30-frame STOI segment (3750 samples at
    10 kHz): NaN STOI / ESTOI and the warning of STOI.py:162-165, on the fast path as on the
    generic one."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(2, 6000, 16000, seed=72, device="cuda")
    m = PESQ_STOI(16000, use_gpu=True)
    assert m._fast_ok(c, n)
    for call in (lambda: m(c, n), lambda: _generic(m, c, n)):
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            res = call()
        assert any("non-silent" in str(x.message) for x in w)
        assert all(d["STOI"] != d["STOI"] and d["PESQ"] == d["PESQ"] for d in res)


def test_scores_written_into_mapped_host_buffer(pairs):
    """fsem_host_buffer_mapped holds for torch's pinned memory on this runtime, so the fast path's
    kernels write the scores straight into the thread's pinned buffer: the buffer holds them after
    the call, and they equal the device-buffer + copy form (host_scores = False) bitwise."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI, _native
    c, n = pairs
    B = c.shape[0]
    m = PESQ_STOI(16000, use_gpu=True)
    assert _native.mapped_host_slot(m, 3 * B) is not None
    res = m(c, n)
    host = m.__dict__["_fsem_tls"].slots[c.device.index][1][:3 * B].reshape(3, B)
    np.testing.assert_array_equal(host[0], np.array([d["PESQ"] for d in res], np.float32))
    np.testing.assert_array_equal(host[2], np.array([d["ESTOI"] for d in res], np.float32))
    cp = PESQ_STOI(16000, use_gpu=True)
    cp.host_scores = False
    assert cp(c, n) == res
    assert not _native.load().fsem_host_buffer_mapped(None)


def test_call_with_scores_fast_path(pairs):
    """call_with_scores (the bench's multi-rank step: the list plus the [B, 3] device scores for the
    all-gather) takes the fast path too: the same list and scores as the generic path, bitwise."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    res, t = m.call_with_scores(c, n)
    m._fast_ok = lambda *a: False
    res_g, t_g = m.call_with_scores(c, n)
    del m._fast_ok
    assert res == res_g
    assert t.shape == (c.shape[0], 3) and t.is_cuda and t.dtype == torch.float32
    np.testing.assert_array_equal(t.cpu().numpy(), t_g.cpu().numpy())
    np.testing.assert_array_equal(t[:, 0].cpu().numpy(), np.array([d["PESQ"] for d in res], np.float32))


@pytest.mark.parametrize("B", [1, 3, 65])
def test_fast_path_small_and_odd_batches(B):
    """The fast path at batch sizes that take the back end's multi-wave forms (B <= 2 per CU) and
    an odd count: the same dicts as the generic path, bitwise, the mapped buffer reused across
    sizes."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(B, 32000, 16000, seed=80 + B, device="cuda")
    m = PESQ_STOI(16000, use_gpu=True)
    assert m._fast_ok(c, n)
    fast = m(c, n)
    assert len(fast) == B and fast == _generic(m, c, n)
    assert m(c[:1], n[:1]) == fast[:1]  # a smaller call after a larger one on the same buffer
