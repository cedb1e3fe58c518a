"""Single-process multi-device fan-out of one metric call ("one stream per device
from a single Python process").

The reference's user scores a batch with one call from one process,
``PESQ_STOI(16000, use_gpu=True)(clean, noisy)`` (``fast_se_metrics/base.py:10-14``,
``benchmark_metrics.py:72-75``), and the reference itself only ever uses the current device.
With ``devices=`` (a list of HIP devices, ``"all"`` or a count) the metric classes split that one
call's rows over several devices instead -- no torch.distributed launch needed:

* rows are cut into contiguous shards, one per listed device, balanced by row count (uniform
  batches) or by summed row length (per-row ``lengths``); utterances are independent, so no data
  moves between shards during compute (the same split as the multi-process path,
  ``distributed.shard_bounds``);
* one host thread and one HIP stream per shard: the thread copies its shard to its device when
  the batch lives elsewhere (point-to-point over xGMI for a batch on another GPU, host-to-device
  for a host batch), scores it with the single-device engine on its stream, and the [k, n] scores
  come back to the first listed device (the metric's device) by one peer copy per shard; a
  shard's input copy from another GPU runs on its own stream of the source device (PyTorch puts
  a device-to-device copy on the source device's current stream: left at the default stream,
  the N-1 shards' copies would queue on one stream, one xGMI link at a time);
* a device may be listed more than once: its shards then run on separate streams of that device
  (the 1-GPU test of this path);
* every stream waits for the caller's stream first (the inputs are ready) and the caller's stream
  waits for every shard (the scores are ready), so ``scores()`` stays asynchronous with respect to
  the host like the single-device call.

Scores equal the single-device call's on the same rows: bitwise for STOI / ESTOI (their sums do
not depend on the batch) and for PESQ whenever the shard and the whole batch use the same PESQ
back-end form (``pesq.hip`` back_waves: one wave per utterance above 2 rows per CU, 4 or 8 below;
the forms differ in summation order only, <= 1e-5 in the MOS, ``tests/test_scale_gpu.py``).
The torch.distributed path (``distributed.py``: one process per GPU, RCCL all-gather) stays the
multi-node / torchrun form.
"""
from __future__ import annotations

import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Sequence

import torch

from .distributed import shard_bounds


def resolve_devices(devices) -> list[torch.device] | None:
    """``devices=`` of the metric constructors -> list of HIP devices, or None (the current
    device only, the reference's behaviour).  Accepts ``"all"`` (every visible device), a count
    n (the first n devices), or a sequence of indices / ``"cuda:i"`` strings / torch.device
    (repeats allowed: several streams on one device)."""
    if devices is None:
        return None
    n_vis = torch.cuda.device_count()
    if isinstance(devices, str) and devices == "all":
        out = [torch.device("cuda", i) for i in range(n_vis)]
    elif isinstance(devices, int) and not isinstance(devices, bool):
        if devices < 1:
            raise ValueError("devices: a count must be >= 1")
        out = [torch.device("cuda", i) for i in range(devices)]
    elif isinstance(devices, (str, torch.device)):
        out = [torch.device(devices)]
    elif isinstance(devices, Sequence):
        out = [torch.device("cuda", d) if isinstance(d, int) else torch.device(d) for d in devices]
    else:
        raise TypeError(f"devices: expected None, 'all', a count or a sequence of devices, got {devices!r}")
    if not out:
        raise ValueError("devices: empty device list")
    for d in out:
        if d.type != "cuda":
            raise ValueError(f"devices: {d} is not a HIP device")
    out = [torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device()) for d in out]
    for d in out:
        if d.index >= n_vis:
            raise ValueError(f"devices: {d} but only {n_vis} HIP device(s) are visible")
    return out


def row_shards(batch: int, n_shards: int, lengths=None) -> list[tuple[int, int]]:
    """Contiguous [lo, hi) row ranges, one per shard: balanced by count (``shard_bounds``) or, with
    per-row lengths, by summed length (the cut after shard k is the row boundary whose running sum
    lies closest to (k+1)/n of the total).  Empty ranges are allowed (fewer rows than shards)."""
    if lengths is None:
        return [shard_bounds(batch, n_shards, k) for k in range(n_shards)]
    cost = torch.as_tensor(lengths).reshape(-1).to("cpu", torch.int64).clamp_min(1)
    csum = [0] + torch.cumsum(cost, 0).tolist()  # csum[j] = rows [0, j)
    total = csum[-1]
    cuts = [0]
    for k in range(1, n_shards):
        target = total * k / n_shards
        j = int(torch.searchsorted(torch.tensor(csum), int(target)))  # first boundary at or past it
        if j > 0 and target - csum[j - 1] <= csum[min(j, batch)] - target:
            j -= 1
        cuts.append(min(max(cuts[-1], j), batch))
    cuts.append(batch)
    return [(cuts[k], max(cuts[k], cuts[k + 1])) for k in range(n_shards)]


_tls = threading.local()


def in_shard() -> bool:
    """True on a FanOut worker thread while it scores its shard (the metric's scores() then runs
    the single-device engine instead of fanning out again)."""
    return getattr(_tls, "active", False)


class FanOut:
    """Host threads + streams of one metric's device list (kept across calls)."""

    # test switch: a shard whose rows already live on its device takes the copy branch anyway (a
    # copy on its copy stream of the source device, ordered by the same events), so the branch of
    # a multi-GPU call runs -- and is checked bitwise -- on a one-GPU box
    force_copy = False

    def __init__(self, devices: list[torch.device]):
        self.devices = devices
        self._pool = ThreadPoolExecutor(max_workers=len(devices), thread_name_prefix="fsem-shard")
        self._streams: list[torch.cuda.Stream | None] = [None] * len(devices)
        self._copy_streams: dict = {}
        self._lock = threading.Lock()
        self.last_copy_streams: list = []

    def _stream(self, k: int) -> torch.cuda.Stream:
        with self._lock:
            if self._streams[k] is None:
                self._streams[k] = torch.cuda.Stream(device=self.devices[k])
            return self._streams[k]

    def _copy_stream(self, k: int, dev: torch.device) -> torch.cuda.Stream:
        """Shard k's stream on the SOURCE device `dev` of its input copy (PyTorch enqueues a
        device-to-device copy on the source device's current stream; in a worker thread that is
        the source's default stream unless set, which would queue every shard's copy on ONE stream
        and so on one xGMI link at a time)."""
        with self._lock:
            key = (k, dev.index)
            st = self._copy_streams.get(key)
            if st is None:
                st = self._copy_streams[key] = torch.cuda.Stream(device=dev)
            return st

    def run(self, score: Callable, clean: torch.Tensor, noisy: torch.Tensor, lengths, ncols: int,
            balance_lengths=None) -> tuple[torch.Tensor, ...]:
        """``score(clean_rows, noisy_rows, lengths_rows) -> tuple of ncols [n] tensors`` on every
        shard -> ncols [B] tensors on the first listed device, in row order, each column in the
        dtype the shards returned it in (float32 scores, int32 time-alignment delays: exact).

        Copies: a shard whose rows live on another GPU pulls them by a peer copy on its own stream
        of the source device (``_copy_stream``: N-1 shards' copies on N-1 streams, hence N-1 xGMI
        links at once), ordered before the shard's compute stream by PyTorch's two-way barrier of
        cross-device copies; each shard writes its scores into the output on its own compute
        stream (a peer copy from the shard's device), and the caller's stream waits for every
        shard's event recorded after that copy.  ``last_copy_streams`` records, per shard, the
        streams its input and output copies ran on (tests/test_multidevice_gpu.py)."""
        B = noisy.shape[0]
        home = self.devices[0]
        bounds = row_shards(B, len(self.devices), balance_lengths)
        caller = torch.cuda.current_stream(home)
        src_dev = noisy.device
        in_ev = None
        if src_dev.type == "cuda":  # the inputs are ready on their device's current stream
            in_ev = torch.cuda.Event()
            in_ev.record(torch.cuda.current_stream(src_dev))
        lens_t = None if lengths is None else torch.as_tensor(lengths).reshape(-1)
        outs: list = [None] * ncols  # allocated on the caller's stream by the first shard to finish
        out_lock = threading.Lock()
        out_ev = torch.cuda.Event()
        copies: list = [None] * len(self.devices)

        def out_cols(cols):
            with out_lock:
                if outs[0] is None:
                    with torch.cuda.stream(caller):  # allocated on (and owned by) the caller's stream
                        for j, t in enumerate(cols):
                            outs[j] = torch.empty(B, dtype=t.dtype, device=home)
                        out_ev.record(caller)
                return list(outs)

        def work(k: int):
            lo, hi = bounds[k]
            if hi <= lo:
                return None
            dev = self.devices[k]
            st = self._stream(k)
            rec = {"compute": st.cuda_stream, "input": None, "output": None}
            with torch.cuda.device(dev), torch.cuda.stream(st):
                if in_ev is not None:
                    st.wait_event(in_ev)
                c, n = clean[lo:hi], noisy[lo:hi]
                if c.device == dev and not self.force_copy:
                    # views of the caller's rows, read on this stream
                    c.record_stream(st)
                    n.record_stream(st)
                    rec["input"] = st.cuda_stream
                elif c.is_cuda:  # peer copy over xGMI on this shard's stream of the source device
                    cs = self._copy_stream(k, c.device)
                    cs.wait_event(in_ev)
                    c.record_stream(cs)
                    n.record_stream(cs)
                    with torch.cuda.stream(cs):
                        if c.device == dev:  # force_copy: the same branch on one device
                            c, n = c.clone(), n.clone()
                        else:
                            c = c.to(dev, non_blocking=True)
                            n = n.to(dev, non_blocking=True)
                        copied = torch.cuda.Event()
                        copied.record(cs)
                    # the shard's stream reads the copies after they land (explicit, beside PyTorch's
                    # own barrier for cross-device copies) and owns them from here on
                    st.wait_event(copied)
                    c.record_stream(st)
                    n.record_stream(st)
                    rec["input"] = cs.cuda_stream
                else:  # host -> device on the shard's stream
                    c = c.to(dev, non_blocking=True)
                    n = n.to(dev, non_blocking=True)
                    rec["input"] = st.cuda_stream
                lk = None
                if lens_t is not None:
                    lk = lens_t[lo:hi]
                    if lk.device != dev:
                        lk = lk.to(dev, non_blocking=True)
                    elif lk.is_cuda:
                        lk.record_stream(st)
                _tls.active = True
                try:
                    cols = score(c, n, lk)
                finally:
                    _tls.active = False
                cols = cols if isinstance(cols, tuple) else (cols,)
                o = out_cols(cols)
                st.wait_event(out_ev)
                # the scores into the output: on this shard's stream (a device-to-device copy runs on
                # the source device's current stream = st), one event after it for the caller
                for j, t in enumerate(cols):
                    o[j][lo:hi].copy_(t, non_blocking=True)
                rec["output"] = torch.cuda.current_stream(dev).cuda_stream
                done = torch.cuda.Event()
                done.record(st)
            copies[k] = rec
            return done

        results = list(self._pool.map(work, range(len(self.devices))))
        for done in results:
            if done is not None:
                caller.wait_event(done)
        self.last_copy_streams = copies
        if outs[0] is None:  # no rows
            return tuple(torch.empty(0, dtype=torch.float32, device=home) for _ in range(ncols))
        return tuple(outs)
