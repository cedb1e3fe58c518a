"""The native list-of-dicts builder behind the drop-in calls (csrc/score_list.c): the same list
the reference's BaseMetric.__call__ returns from tensor.tolist() (fast_se_metrics/base.py), for
float32 and float64 scores, empty batches and NaN; malformed input raises."""
import math

import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import _native


def _py(t, keys):
    return [dict(zip(keys, r)) for r in zip(*t.tolist())]


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_matches_tolist(dtype):
    g = torch.Generator().manual_seed(0)
    t = torch.randn(3, 1000, generator=g, dtype=dtype)
    t[1, 7] = float("nan")
    t[0, 3] = float("inf")
    keys = ("PESQ", "STOI", "ESTOI")
    got = _native.score_list(t, keys)
    ref = _py(t, keys)
    assert len(got) == len(ref) == 1000
    for a, b in zip(got, ref):
        assert list(a) == list(keys)
        for k in keys:
            assert (math.isnan(a[k]) and math.isnan(b[k])) or a[k] == b[k]
            assert type(a[k]) is float


def test_single_key_and_empty():
    assert _native.score_list(torch.tensor([[1.5, 2.0]]), ("PESQ",)) == [{"PESQ": 1.5}, {"PESQ": 2.0}]
    assert _native.score_list(torch.empty(2, 0), ("STOI", "ESTOI")) == []
    assert _native.score_list(np.zeros((2, 0), np.float32), ("STOI", "ESTOI")) == []


def test_rejects_bad_input():
    with pytest.raises(TypeError):
        _native.score_list(np.zeros((3, 4), np.int32), ("a", "b", "c"))
    with pytest.raises(TypeError):
        _native.score_list(np.zeros(5, np.float32), ("a", "b", "c"))  # 5 values, 3 keys
    with pytest.raises(ValueError):
        _native.score_list(np.zeros((1, 4), np.float32), ())
    with pytest.raises(TypeError):
        _native.score_list(np.zeros((1, 4), np.float32), (1,))


@pytest.fixture
def python_builder(monkeypatch):
    """The native builder unavailable (as without a C compiler / Python headers / a writable
    package directory): _native.score_list takes the Python form."""
    monkeypatch.setattr(_native, "_score_list_mod", False)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_python_fallback_matches_native(dtype, python_builder):
    g = torch.Generator().manual_seed(1)
    t = torch.randn(3, 257, generator=g, dtype=dtype)
    t[2, 5] = float("nan")
    keys = ("PESQ", "STOI", "ESTOI")
    got = _native.score_list(t, keys)
    want = _py(t, keys)
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert list(a) == list(keys)
        for k in keys:
            assert (math.isnan(a[k]) and math.isnan(b[k])) or a[k] == b[k]
            assert type(a[k]) is float


def test_python_fallback_checks(python_builder):
    assert _native.score_list(torch.tensor([[1.5, 2.0]]), ("PESQ",)) == [{"PESQ": 1.5}, {"PESQ": 2.0}]
    assert _native.score_list(np.zeros((2, 0), np.float32), ("STOI", "ESTOI")) == []
    with pytest.raises(TypeError):
        _native.score_list(np.zeros((3, 4), np.int32), ("a", "b", "c"))
    with pytest.raises(TypeError):
        _native.score_list(np.zeros(5, np.float32), ("a", "b", "c"))
    with pytest.raises(ValueError):
        _native.score_list(np.zeros((1, 4), np.float32), ())
    with pytest.raises(TypeError):
        _native.score_list(np.zeros((1, 4), np.float32), (1,))


def test_drop_in_call_without_native_builder(python_builder):
    """The CPU-mode drop-in call works (same list) when the native builder cannot be built."""
    from fast_speech_enhancement_metrics_amd import STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(2, 16000, 10000, seed=3)
    s, e = STOI(10000).scores(c, n)
    got = STOI(10000)(c, n)
    assert got == [{"STOI": float(a), "ESTOI": float(b)} for a, b in zip(s.float().tolist(), e.float().tolist())]


def test_unbuildable_native_builder_falls_back(monkeypatch):
    """A failing build (e.g. no C compiler) warns once and leaves the Python form in place."""
    from fast_speech_enhancement_metrics_amd import _build

    def broken(*a, **k):
        raise RuntimeError("no C compiler found")

    monkeypatch.setattr(_native, "_score_list_mod", None)
    monkeypatch.setattr(_build, "build_score_list", broken)
    with pytest.warns(RuntimeWarning, match="native score-list builder unavailable"):
        got = _native.score_list(np.array([[1.0, 2.0]], np.float32), ("PESQ",))
    assert got == [{"PESQ": 1.0}, {"PESQ": 2.0}]
    assert _native._score_list_mod is False


@pytest.fixture(params=["native", "python"])
def builder(request, monkeypatch):
    if request.param == "python":
        monkeypatch.setattr(_native, "_score_list_mod", False)
    return request.param


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_alloc_fill_matches_score_list(dtype, builder):
    """The GPU path's two-phase form (dicts built before the scores exist, filled per chunk)
    returns the list score_list builds: same keys in order, same float values, NaN included."""
    g = torch.Generator().manual_seed(2)
    t = torch.randn(3, 300, generator=g, dtype=dtype)
    t[1, 7] = float("nan")
    keys = ("PESQ", "STOI", "ESTOI")
    lst, h = _native.score_list_alloc(300, keys)
    assert len(lst) == 300 and all(list(d) == list(keys) and all(math.isnan(v) for v in d.values()) for d in lst)
    for lo, hi in ((120, 300), (0, 120)):  # chunks, in any order
        _native.score_list_fill(h, lo, t[:, lo:hi].contiguous(), keys)
    del h
    want = _py(t, keys)
    for a, b in zip(lst, want):
        assert list(a) == list(keys)
        for k in keys:
            assert (math.isnan(a[k]) and math.isnan(b[k])) or a[k] == b[k]
            assert type(a[k]) is float
    assert _native.score_list_alloc(0, keys)[0] == []


def test_fill_leaves_shared_objects_alone(builder):
    """A float the caller holds is replaced, never written in place; dicts the caller changed
    still get every key."""
    keys = ("STOI", "ESTOI")
    lst, h = _native.score_list_alloc(3, keys)
    held = lst[0]["STOI"]
    lst[1]["extra"] = 1.0
    del lst[2]["STOI"]
    _native.score_list_fill(h, 0, np.array([[0.5, 0.25, 0.125], [1.0, 2.0, 3.0]], np.float32), keys)
    assert math.isnan(held)
    assert lst[0] == {"STOI": 0.5, "ESTOI": 1.0}
    assert lst[1] == {"STOI": 0.25, "ESTOI": 2.0, "extra": 1.0}
    assert lst[2] == {"STOI": 0.125, "ESTOI": 3.0}
    del h
    import sys
    for d in lst:  # the handle's references are gone: only the dicts' (+ getrefcount's argument)
        refs = [sys.getrefcount(d[k]) for k in keys]  # outside the assert (its rewrite holds temporaries)
        assert refs == [2] * len(keys)


def test_fill_rejects_bad_input(builder):
    keys = ("PESQ",)
    _, h = _native.score_list_alloc(2, keys)
    with pytest.raises(IndexError):
        _native.score_list_fill(h, 1, np.zeros((1, 2), np.float32), keys)
    with pytest.raises(TypeError):
        _native.score_list_fill(h, 0, np.zeros((1, 2), np.int32), keys)
    with pytest.raises(ValueError):
        _native.score_list_fill(h, 0, np.zeros((2, 2), np.float32), ("PESQ", "STOI"))
    with pytest.raises(ValueError):
        _native.score_list_alloc(2, ())


def test_fill_rejects_mismatched_keys_of_equal_count(builder):
    """Both builders refuse keys that differ from the allocation's in any element (the native
    in-place path writes through the allocation's float objects, so a different key tuple of the
    same length must not be accepted); equal keys in a new tuple object are fine."""
    keys = ("STOI", "ESTOI")
    lst, h = _native.score_list_alloc(2, keys)
    scores = np.array([[0.5, 0.25], [1.0, 2.0]], np.float32)
    for bad in (("ESTOI", "STOI"), ("STOI", "PESQ"), ("PESQ", "ESTOI")):
        with pytest.raises(ValueError, match="keys differ"):
            _native.score_list_fill(h, 0, scores, bad)
    assert all(math.isnan(v) for d in lst for v in d.values())  # nothing written by the refused calls
    _native.score_list_fill(h, 0, scores, tuple(["STOI", "E" + "STOI"]))
    assert lst == [{"STOI": 0.5, "ESTOI": 1.0}, {"STOI": 0.25, "ESTOI": 2.0}]


def test_fill_dict_path_equals_inplace_path():
    """score_list_fill writes fresh floats in place only on GIL builds of CPython <= 3.13 (VERDICT
    r5 item 5: it relies on their refcount semantics); elsewhere, and with set_inplace(False),
    every value goes through PyDict_SetItem.  Both forms give the same list, also for rows the
    caller touched in between."""
    import sys
    import sysconfig
    mod = _native._load_score_list()
    assert mod is not False
    free_threaded = bool(sysconfig.get_config_var("Py_GIL_DISABLED"))
    assert mod.INPLACE_COMPILED == int(not free_threaded and sys.version_info < (3, 14))
    g = torch.Generator().manual_seed(5)
    t = torch.randn(3, 257, generator=g).numpy()
    t[2, 9] = float("nan")
    keys = ("PESQ", "STOI", "ESTOI")
    lists = []
    for inplace in (True, False):
        prev = mod.set_inplace(inplace)
        try:
            lst, h = _native.score_list_alloc(257, keys)
            held = lst[4]["STOI"]  # a value the caller holds: filled by a new float either way
            _native.score_list_fill(h, 0, t[:, :100].copy(), keys)
            _native.score_list_fill(h, 100, t[:, 100:].copy(), keys)
            assert math.isnan(held)
            lists.append(lst)
        finally:
            mod.set_inplace(prev)
    ref = _py(torch.from_numpy(t), keys)
    for lst in lists:
        assert len(lst) == 257
        for a, b in zip(lst, ref):
            for k in keys:
                assert (math.isnan(a[k]) and math.isnan(b[k])) or a[k] == b[k]
    assert mod.set_inplace(True) == bool(mod.INPLACE_COMPILED)
