"""What a metric keeps between drop-in calls is process state: the per-thread pinned
score buffers (a threading.local), the last result list's fill handle (a PyCapsule) and the
fan-out's threads.  Copies and pickles of a metric drop it -- the reference's BaseMetric
(fast_se_metrics/base.py:6-43) is a plain object that can be copied -- and release() frees it."""
import copy
import pickle
import threading

import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI, _native


@pytest.mark.parametrize("cls", [PESQ, STOI, PESQ_STOI])
def test_copy_and_pickle_drop_call_state(cls):
    m = cls(16000, use_gpu=False)
    # what a GPU call leaves behind (a native fill handle is a PyCapsule: neither copyable nor picklable)
    m.__dict__["_fsem_tls"] = threading.local()
    m.__dict__["_fsem_tls"].slots = {0: (torch.zeros(4),)}
    m.__dict__["_held_list"] = _native.score_list_alloc(2, ("PESQ",))[1]
    for c in (copy.deepcopy(m), pickle.loads(pickle.dumps(m)), copy.copy(m)):
        assert "_fsem_tls" not in c.__dict__ and "_held_list" not in c.__dict__
        assert c._fanout is None and c.sample_rate == 16000 and type(c) is cls
    # the copy scores as the original
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 16000, generator=g)
    y = x + 0.1 * torch.randn(2, 16000, generator=g)
    c = pickle.loads(pickle.dumps(m))
    assert c(x, y) == cls(16000, use_gpu=False)(x, y)


def test_release_drops_held_list_and_slots():
    m = PESQ_STOI(16000, use_gpu=False)
    m.release()  # nothing held yet: a no-op
    m.__dict__["_fsem_tls"] = threading.local()
    m.__dict__["_fsem_tls"].slots = {0: (torch.zeros(4),)}
    m.__dict__["_held_list"] = object()
    m.release()
    assert "_held_list" not in m.__dict__ and m.__dict__["_fsem_tls"].slots == {}
