"""Concurrent callers on one GPU: the C-ABI is re-entrant across streams and host threads
(include/fsem.h conventions).  The engine enqueues on the caller's current stream; the joint entry
and the PESQ entry also run the back end on a per-device side stream joined back into the caller's
stream (pesq.hip side_stream / stream_wait, one join event per host thread), so concurrent calls on
different streams share that side stream.  Every score must equal the serial default-stream result
bitwise -- including when the caller's inputs, workspace and outputs are freed and reused by the
caching allocator right after each call -- and the caller's stream alone must order the results
(no device-wide synchronisation before reading them on that stream).
"""
import threading

import pytest
import torch

pytestmark = pytest.mark.gpu

L = 48000  # 3 s @ 16 kHz
SIZES = (3, 200, 600)  # PESQ back end over 8 / 4 / 1 waves per utterance (pesq.hip launch_back: up to half
                       # a row per CU / up to 2 rows per CU / above)


@pytest.fixture(scope="module")
def work():
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    metrics = {"pesq": PESQ(16000, use_gpu=True), "stoi": STOI(16000, use_gpu=True),
               "joint": PESQ_STOI(16000, use_gpu=True)}
    batches = [speech_like_pairs(B, L, 16000, seed=100 + i, device="cuda")[:2] for i, B in enumerate(SIZES)]

    def run(kind, c, n):
        m = metrics[kind]
        if kind == "pesq":
            return (m.scores(c, n),)
        if kind == "stoi":
            return m.scores(c, n, 16000)
        return m.scores(c, n)

    ref = {(k, i): [t.clone() for t in run(k, c, n)] for k in metrics for i, (c, n) in enumerate(batches)}
    torch.cuda.synchronize()
    return run, batches, ref


def _same(a, b):
    """Bitwise equal, NaN in the same places."""
    return all(torch.equal(torch.isnan(x).cpu(), torch.isnan(y).cpu()) and
               torch.equal(x.nan_to_num().cpu(), y.nan_to_num().cpu()) for x, y in zip(a, b))


def test_non_default_stream_matches_default(work):
    run, batches, ref = work
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        out = {(k, i): run(k, c, n) for k in ("pesq", "stoi", "joint") for i, (c, n) in enumerate(batches)}
        host = {key: [t.cpu() for t in v] for key, v in out.items()}  # ordered by s alone
    for key, v in host.items():
        assert _same(v, ref[key]), key


def test_threads_on_own_streams_match_serial(work):
    run, batches, ref = work
    errors, results = [], {}
    start = threading.Barrier(3)

    def worker(tid):
        try:
            s = torch.cuda.Stream()
            start.wait()
            with torch.cuda.stream(s):
                for rep in range(4):
                    for j in range(len(batches)):
                        i = (j + tid + rep) % len(batches)
                        kind = ("pesq", "stoi", "joint")[(tid + rep + j) % 3]
                        c, n = batches[i]
                        # fresh copies made on this stream: their blocks are recycled by the caching
                        # allocator between calls, as a serving loop's would be
                        cc, nn = c.clone(), n.clone()
                        out = run(kind, cc, nn)
                        del cc, nn
                        results[(tid, rep, j)] = (kind, i, [t.cpu() for t in out])
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(repr(e))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in threads), "worker threads did not finish"
    assert not errors, errors
    assert len(results) == 3 * 4 * len(batches)
    for key, (kind, i, out) in results.items():
        assert _same(out, ref[(kind, i)]), (key, kind, i)
