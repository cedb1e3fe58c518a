"""ctypes binding of libfsem.so (include/fsem.h), the gfx950 HIP engine.

The library is loaded AFTER torch so that its ``libamdhip64.so.7`` dependency resolves to
the HIP runtime torch already loaded (one runtime per process: torch's streams and device
pointers are valid in the library).  There is no fallback: if the library is missing or
cannot be loaded, every GPU entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_PKG, "lib", "libfsem.so")
LIB_PATH = os.environ.get("FSEM_LIB", _DEFAULT_LIB)

FSEM_OK = 0
FSEM_EINVAL = -1
FSEM_EWORKSPACE = -2
FSEM_ELAUNCH = -3
FSEM_ESHORT = -4
FSEM_ERATE = -5

_lock = threading.Lock()
_lib = None

_c_i64 = ctypes.c_int64
_c_i32 = ctypes.c_int32
_c_sz = ctypes.c_size_t
_vp = ctypes.c_void_p

# name -> (restype, argtypes); every symbol include/fsem.h declares
SIGNATURES = {
    "fsem_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "fsem_version": (ctypes.c_int, []),
    "fsem_build_id": (ctypes.c_char_p, []),
    "fsem_host_buffer_mapped": (ctypes.c_int, [ctypes.c_void_p]),
    "fsem_resample_length": (_c_i64, [_c_i64, _c_i32, _c_i32]),
    "fsem_resample_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _c_i32, _c_i32, _vp]),
    "fsem_resample_rows_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _c_i32, _c_i32, _vp]),
    "fsem_pesq_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_frames": (ctypes.c_int, [_c_i64]),
    "fsem_pesq_wb_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_pesq_front_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_front_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_pesq_front_y10_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_i64,
                                                _vp, _c_i64, _vp, _c_sz, _vp]),
    "fsem_pesq_back_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_back_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_pre_emphasize_f32": (ctypes.c_int, [_vp, _c_i64, _c_i64, _c_i64, _vp, _c_i64, _vp]),
    "fsem_pesq_distances_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_distances_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_stoi_workspace_bytes": (_c_sz, [_c_i64, _c_i64, _c_i32]),
    "fsem_stoi_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i32, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_stoi_tob_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _c_i64, _vp, _c_sz, _vp]),
    "fsem_pesq_stoi_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_stoi_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_sz, _vp]),
    "fsem_time_align_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_time_align_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i32, _vp, _vp, _c_i64, _vp,
                                            _c_sz, _vp]),
    "fsem_time_align_utt_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_time_align_p862_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_time_align_p862_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i32, _vp, _vp, _vp, _vp,
                                                 _vp, _c_i64, _vp, _c_sz, _vp]),
    "fsem_time_align_utt_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _c_i32, _vp, _vp, _vp, _vp,
                                                _vp, _c_i64, _vp, _c_sz, _vp]),
    "fsem_pesq_bad_intervals_workspace_bytes": (_c_sz, [_c_i64, _c_i64]),
    "fsem_pesq_bad_intervals_f32": (ctypes.c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp,
                                                    _vp, _vp, _vp, _c_i64, _vp, _c_sz, _vp]),
    "fsem_pesq_pool_f32": (ctypes.c_int, [_vp, _vp, _vp, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp]),
    "fsem_pesq_wb_frames_f32": (ctypes.c_int, [_vp, _vp, _c_i64, _c_i64, _c_i64, _vp, _vp, _vp, _vp, _vp, _c_sz,
                                               _vp]),
}
ALIGN_MAX_SEGMENTS = 32  # include/fsem.h FSEM_ALIGN_MAX_SEGMENTS
PESQ_MAX_BAD = 16  # include/fsem.h FSEM_PESQ_MAX_BAD


_score_list_mod = None  # the native builder's module; False: unavailable, the Python form is used


def score_list_py(scores, keys: tuple) -> list:
    """Python form of the native list builder (same result, same argument checks): a dict per
    column of the [K, B] float32 / float64 scores."""
    if not isinstance(keys, tuple):
        raise TypeError("score_list: keys must be a tuple")
    if not keys:
        raise ValueError("score_list: keys must be a non-empty tuple")
    if not all(isinstance(k, str) for k in keys):
        raise TypeError("score_list: keys must be str")
    import numpy as np
    a = np.asarray(scores)
    if a.dtype not in (np.float32, np.float64) or a.size % len(keys):
        raise TypeError("score_list: scores must be a contiguous float32 / float64 buffer of K x B values")
    return [dict(zip(keys, col)) for col in zip(*a.reshape(len(keys), -1).tolist())]


def _load_score_list():
    """The native builder (csrc/score_list.c, compiled by _build.build_score_list on first use if
    absent), or False where it cannot be built or loaded -- no C compiler or Python headers, a
    read-only package directory, FSEM_SCORE_LIST=python: the drop-in calls then build their lists
    in Python (score_list_py), with a warning once."""
    global _score_list_mod
    with _lock:
        if _score_list_mod is None:
            if os.environ.get("FSEM_SCORE_LIST") == "python":
                _score_list_mod = False
                return False
            try:
                import importlib.machinery
                import importlib.util

                from . import _build
                path = _build.build_score_list()
                loader = importlib.machinery.ExtensionFileLoader("_score_list", path)
                spec = importlib.util.spec_from_file_location("_score_list", path, loader=loader)
                m = importlib.util.module_from_spec(spec)
                loader.exec_module(m)
                _score_list_mod = m
            except Exception as exc:  # noqa: BLE001 -- any build / load failure: the Python form
                import warnings
                warnings.warn(f"native score-list builder unavailable ({exc!r}); building result lists in Python",
                              RuntimeWarning, stacklevel=3)
                _score_list_mod = False
    return _score_list_mod


def score_list(scores, keys: tuple) -> list:
    """[{keys[k]: scores[k][b]} for b in range(B)] from a C-contiguous float32 [K, B] host array
    (numpy, or a CPU tensor) -- the drop-in call's result list, built natively
    (csrc/score_list.c), or by score_list_py where the native builder is unavailable."""
    mod = _score_list_mod
    if mod is None:
        mod = _load_score_list()
    if isinstance(scores, torch.Tensor):
        scores = scores.detach().cpu().contiguous().numpy()
    if mod is False:
        return score_list_py(scores, keys)
    return mod.score_list(scores, keys)


def score_list_alloc(n: int, keys: tuple):
    """The drop-in call's result list before its scores are known: (list of n dicts over `keys`
    with NaN values, handle) -- built while the GPU computes; score_list_fill(handle, ...)
    writes the scores into the list."""
    mod = _score_list_mod
    if mod is None:
        mod = _load_score_list()
    if mod is False:
        score_list_py(_np_empty(len(keys), 0), keys)  # the same argument checks
        lst = [dict.fromkeys(keys, float("nan")) for _ in range(n)]
        return lst, (lst, keys)
    return mod.score_list_alloc(n, keys)


def score_list_fill(handle, offset: int, scores, keys: tuple) -> None:
    """list[offset + b][keys[k]] = scores[k][b] for the [K, B] host scores (numpy or a CPU tensor)
    and the list of score_list_alloc's handle: the same dicts and values as
    score_list(scores, keys) at list[offset:offset + B]."""
    mod = _score_list_mod
    if mod is None:
        mod = _load_score_list()
    if isinstance(scores, torch.Tensor):
        scores = scores.detach().cpu().contiguous().numpy()
    if mod is False:
        lst, akeys = handle
        if tuple(keys) != akeys:
            raise ValueError("score_list_fill: keys differ from the allocation's")
        rows = score_list_py(scores, keys)
        if offset < 0 or offset + len(rows) > len(lst):
            raise IndexError("score_list_fill: rows past the list's end")
        for b, row in enumerate(rows):
            lst[offset + b].update(row)
        return
    mod.score_list_fill(handle, offset, scores, keys)


def _host_slot(owner, n: int, device):
    """(pinned float32 host buffer of >= n elements, its numpy view, an event) of `owner` (a metric),
    this host thread and `device`, kept across calls: a drop-in call waits for its copy before
    returning, so the next call on the thread may reuse them.  Keyed by device: an event belongs
    to the device of its first record, and whether the device maps the buffer
    (fsem_host_buffer_mapped) is a property of that device."""
    tl = owner.__dict__.get("_fsem_tls")
    if tl is None:
        tl = owner.__dict__.setdefault("_fsem_tls", threading.local())
    slots = getattr(tl, "slots", None)
    if slots is None:
        slots = tl.slots = {}
    idx = torch.device(device).index
    if idx is None:
        idx = torch.cuda.current_device()
    slot = slots.get(idx)
    if slot is None or slot[0].numel() < n:
        buf = torch.empty(max(n, 3 * 4096), dtype=torch.float32, pin_memory=True)
        with torch.cuda.device(idx):
            mapped = bool(load().fsem_host_buffer_mapped(buf.data_ptr()))
            ev = torch.cuda.Event()
        slot = slots[idx] = (buf, buf.numpy(), ev, mapped)
    buf, buf_np, ev, _ = slot
    return buf[:n], buf_np[:n], ev


def mapped_host_slot(owner, n: int, device=None):
    """`owner`'s pinned host buffer for this thread and `device` (as _host_slot) when that device
    may write it directly (fsem_host_buffer_mapped: the same address on host and device), else
    None."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    pin, pin_np, ev = _host_slot(owner, n, device)
    idx = torch.device(device).index
    return (pin, pin_np, ev) if owner.__dict__["_fsem_tls"].slots[idx][3] else None


def list_from_host(owner, slot, K: int, B: int, keys: tuple, device):
    """list_from_device for scores the kernels write straight into `slot` (mapped_host_slot):
    no copy behind the kernels, only the event on the current stream."""
    _, pin_np, ev = slot
    ev.record(torch.cuda.current_stream(device))
    owner._held_list = None
    res, h = score_list_alloc(B, keys)
    ev.synchronize()
    host = pin_np[:K * B].reshape(K, B)
    score_list_fill(h, 0, host, keys)
    owner._held_list = h
    return res, host


def release(owner) -> None:
    """Drop what a metric keeps between drop-in calls: the last result list's fill handle and this
    host thread's pinned score buffers (BaseMetric.release)."""
    owner.__dict__.pop("_held_list", None)
    tl = owner.__dict__.get("_fsem_tls")
    if tl is not None and getattr(tl, "slots", None):
        tl.slots = {}


def list_from_device(owner, t: torch.Tensor, keys: tuple):
    """The drop-in call's result list from [K, B] float32 scores on the GPU, (list, host scores
    [K, B] numpy).  Enqueues the scores' copy into pinned host memory behind the kernels on the
    current stream, then -- while the GPU computes -- releases the list `owner` returned last
    time and builds the new list's dicts (score_list_alloc); fills them when the copy has landed
    and keeps the new list (through its fill handle) until `owner`'s next call.  The list a
    caller drops is then freed during the next call's kernels instead of between two calls, when
    the GPU would wait for it (4096 dicts: ~0.1-0.2 ms of deallocation)."""
    K, B = t.shape
    pin, pin_np, ev = _host_slot(owner, K * B, t.device)
    pin.view(K, B).copy_(t, non_blocking=True)
    ev.record(torch.cuda.current_stream(t.device))
    owner._held_list = None  # the previous call's list, released while the GPU computes
    res, h = score_list_alloc(B, keys)
    ev.synchronize()
    host = pin_np.reshape(K, B)
    score_list_fill(h, 0, host, keys)
    owner._held_list = h  # (the handle holds the list, hence its dicts and floats)
    return res, host


def _np_empty(k: int, n: int):
    import numpy as np
    return np.empty((k, n), dtype=np.float32)


class NativeError(RuntimeError):
    pass


def _check_build_id() -> None:
    """The in-tree library must be the build of this tree's sources and flags (_build.source_hash,
    embedded as fsem_build_id()) for this process's target (_build.ARCH, FSEM_OFFLOAD_ARCH):

    * built for another target -> ImportError, never a rebuild (a gfx942 build loaded by a
      process that did not set FSEM_OFFLOAD_ARCH is not silently replaced by a gfx950 one);
    * stale (other sources or flags) -> ImportError, unless FSEM_AUTOBUILD=1 opts in to a rebuild
      with hipcc (so the ranks of a multi-process job do not each run hipcc at import);

    no kernel runs from a binary the committed sources did not produce.  FSEM_LIB (a library
    variant chosen explicitly, tools/ab_*.py) is not checked."""
    if LIB_PATH != _DEFAULT_LIB:
        return
    from . import _build
    if not all(os.path.exists(d) for d in _build.deps()):
        return  # no source tree next to the package (nothing to compare with)
    arch = _build.library_build_arch(LIB_PATH)
    if arch != _build.ARCH:
        raise ImportError(f"fsem HIP engine {LIB_PATH} was built for {arch}, this process targets {_build.ARCH} "
                          "(FSEM_OFFLOAD_ARCH): rebuild it with `python -m fast_speech_enhancement_metrics_amd._build`")
    want = _build.source_hash()
    have = _build.library_build_id(LIB_PATH)
    if have == want:
        return
    if os.environ.get("FSEM_AUTOBUILD") != "1":
        raise ImportError(f"fsem HIP engine {LIB_PATH} is stale (build id {have}, sources {want}): rebuild it with "
                          "`python -m fast_speech_enhancement_metrics_amd._build` (or set FSEM_AUTOBUILD=1)")
    try:
        _build.build(force=True)
    except Exception as exc:  # noqa: BLE001 -- any build failure: refuse the stale binary
        raise ImportError(f"fsem HIP engine {LIB_PATH} is stale (build id {have}, sources {want}) and could not "
                          f"be rebuilt: {exc!r}") from exc
    have = _build.library_build_id(LIB_PATH)
    if have != want:
        raise ImportError(f"fsem HIP engine {LIB_PATH}: build id {have} after rebuilding, sources {want}")


def build_id() -> str:
    """The loaded library's build id (fsem_build_id())."""
    return load().fsem_build_id().decode()


def load() -> ctypes.CDLL:
    """Load (once) and return the library; raises if it is missing or stale."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"fsem HIP engine not built: {LIB_PATH} is missing "
                    "(run `python -m fast_speech_enhancement_metrics_amd._build`)")
            _check_build_id()
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int, what: str) -> None:
    if rc != FSEM_OK:
        msg = load().fsem_strerror(rc).decode()
        raise NativeError(f"{what}: {msg} ({rc})")


def stream_handle(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


def workspace(nbytes: int, device) -> torch.Tensor:
    """Scratch from torch's caching allocator (cheap after the first call)."""
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)
