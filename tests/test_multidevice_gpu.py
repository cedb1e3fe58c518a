"""Single-process multi-device drop-in call (multidevice.py, SURVEY 8(e) "one stream per device
from a single Python process").  On the 1-GPU box the device list repeats
cuda:0, so two (or three) shards run on separate streams of one device, each in its own host
thread: the scores equal the single-device call's bitwise -- STOI / ESTOI always, PESQ where shard
and batch use the same back-end form (batches here stay in the 8-wave class, pesq.hip back_waves)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pairs():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(24, 48000, 16000, seed=61, device="cuda")
    return c, n


def _np(ts):
    return [t.cpu().numpy() for t in ts]


@pytest.mark.parametrize("devices", [["cuda:0", "cuda:0"], [0, 0, 0]])
def test_joint_scores_equal_single_device(pairs, devices):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    one = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n))
    m = PESQ_STOI(16000, use_gpu=True, devices=devices)
    got = m.scores(c, n)
    assert all(t.device == torch.device("cuda", 0) for t in got)
    for a, b in zip(_np(got), one):
        np.testing.assert_array_equal(a, b)
    # the drop-in call: one list of dicts in row order
    res = m(c, n)
    assert len(res) == c.shape[0]
    np.testing.assert_array_equal(np.array([d["PESQ"] for d in res], np.float32), one[0])
    np.testing.assert_array_equal(np.array([d["STOI"] for d in res], np.float32), one[1])
    np.testing.assert_array_equal(np.array([d["ESTOI"] for d in res], np.float32), one[2])


def test_host_inputs_and_separate_metrics(pairs):
    """Inputs on the host: each shard copies its own rows to its device (no staging copy of the
    whole batch); PESQ and STOI alone fan out alike."""
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    c, n = pairs
    ch, nh = c.cpu(), n.cpu()
    want_p = PESQ(16000, use_gpu=True).scores(c, n).cpu().numpy()
    want_s = _np(STOI(16000, use_gpu=True).scores(c, n, 16000))
    p = PESQ(16000, use_gpu=True, devices=["cuda:0", "cuda:0"])
    np.testing.assert_array_equal(p.scores(ch, nh).cpu().numpy(), want_p)
    assert [d["PESQ"] for d in p(ch, nh)] == want_p.tolist()
    s = STOI(16000, use_gpu=True, devices=["cuda:0", "cuda:0"])
    for a, b in zip(_np(s.scores(ch, nh, 16000)), want_s):
        np.testing.assert_array_equal(a, b)
    got = s(ch, nh)
    np.testing.assert_array_equal(np.array([d["STOI"] for d in got], np.float32), want_s[0])


def test_ragged_rows_balanced_by_length(pairs):
    """Per-row lengths: shards are cut by summed length; every row scores as the single-device call."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    g = np.random.default_rng(3)
    lens = torch.from_numpy(g.integers(6000, 48001, c.shape[0]).astype(np.int32)).cuda()
    one = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n, lengths=lens))
    got = _np(PESQ_STOI(16000, use_gpu=True, devices=[0, 0]).scores(c, n, lengths=lens))
    for a, b in zip(got, one):
        np.testing.assert_array_equal(a, b)


def test_other_rate_and_time_alignment(pairs):
    """8 kHz rows (PESQ 8->16 kHz, STOI 8->10 kHz per shard) and PESQ with each time-alignment
    mode (row, utterance, P.862 with its bad-interval rescoring per shard): delays and scores
    reassembled in row order, bitwise the single-device call's."""
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c8, n8, _ = speech_like_pairs(10, 24000, 8000, seed=62, device="cuda")
    one = _np(PESQ_STOI(8000, use_gpu=True).scores(c8, n8, sample_rate=8000))
    got = _np(PESQ_STOI(8000, use_gpu=True, devices=[0, 0]).scores(c8, n8, sample_rate=8000))
    for a, b in zip(got, one):
        np.testing.assert_array_equal(a, b)
    c, n = pairs
    D = torch.arange(c.shape[0], device="cuda") * 37 - 400
    t = torch.arange(c.shape[1], device="cuda")
    src = t[None, :] - D[:, None]
    deg = torch.where((src >= 0) & (src < c.shape[1]), n.gather(1, src.clamp(0, c.shape[1] - 1)), torch.zeros_like(n))
    for mode in (True, "utterance", "p862"):
        a1 = PESQ(16000, use_gpu=True, time_align=mode)
        want = a1.scores(c, deg).cpu().numpy()
        a2 = PESQ(16000, use_gpu=True, time_align=mode, devices=[0, 0])
        np.testing.assert_array_equal(a2.scores(c, deg).cpu().numpy(), want)
        np.testing.assert_array_equal(a2.last_delays.cpu().numpy(), a1.last_delays.cpu().numpy())


def test_streams_overlap_and_caller_stream_order(pairs):
    """The call is asynchronous for the host; results consumed on the caller's stream are complete
    (the caller's stream waits for every shard), also from a non-default caller stream."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    want = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n))
    m = PESQ_STOI(16000, use_gpu=True, devices=[0, 0])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream())
        outs = [m.scores(c, n) for _ in range(3)]
        summed = [sum(o[j] for o in outs) for j in range(3)]
    s.synchronize()
    for j in range(3):
        np.testing.assert_array_equal(summed[j].cpu().numpy(), 3 * want[j])


def test_copy_streams_per_shard(pairs):
    """Copy placement: each shard's copies run on streams of its own -- never
    all on one stream of the source device.  On the 1-GPU box: the output copies of the shards run
    on the shards' own compute streams (distinct per shard, none the caller's or the default
    stream), host inputs are copied on those streams too, and the per-shard source-device copy
    streams (the peer-copy path of a batch held by another GPU) are distinct per shard."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True, devices=[0, 0, 0])
    want = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n))
    caller = torch.cuda.current_stream().cuda_stream
    default = torch.cuda.default_stream().cuda_stream
    for inputs in ((c, n), (c.cpu(), n.cpu())):
        got = _np(m.scores(*inputs))
        for a, b in zip(got, want):
            np.testing.assert_array_equal(a, b)
        rec = m._fanout.last_copy_streams
        assert len(rec) == 3 and all(r is not None for r in rec)
        outs = [r["output"] for r in rec]
        assert len(set(outs)) == 3 and caller not in outs and default not in outs
        assert all(r["output"] == r["compute"] == r["input"] for r in rec)
    fo = m._fanout
    dev0 = torch.device("cuda", 0)
    cs = [fo._copy_stream(k, dev0) for k in range(3)]
    assert len({s.cuda_stream for s in cs}) == 3 and default not in {s.cuda_stream for s in cs}
    assert fo._copy_stream(1, dev0) is cs[1]  # kept across calls


def test_home_device_current_for_resampling(pairs):
    """A multi-device metric resamples its rows on its home device with that device current
    (the engine launches on the current HIP device); 8 kHz rows through devices=[0, 0]
    from inside another device context still score as the single-device call."""
    from fast_speech_enhancement_metrics_amd import PESQ
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c8, n8, _ = speech_like_pairs(6, 24000, 8000, seed=63, device="cuda")
    want = PESQ(8000, use_gpu=True)(c8, n8)
    m = PESQ(8000, use_gpu=True, devices=[0, 0])
    with torch.cuda.device(0):
        got = m(c8, n8)
    assert [d["PESQ"] for d in got] == [d["PESQ"] for d in want]


def test_time_alignment_delays_keep_int32_through_fanout(pairs):
    """Delays come back through the fan-out in int32 (exact beyond 2^24 samples)."""
    from fast_speech_enhancement_metrics_amd.multidevice import FanOut
    fo = FanOut([torch.device("cuda", 0)] * 2)
    big = torch.tensor([2 ** 24 + 1, 2 ** 29 - 3, -(2 ** 25) - 1, 7], dtype=torch.int32, device="cuda")
    c = torch.zeros(4, 8, device="cuda")

    def score(cc, nn, lk):
        lo = int(cc[:, 0].numel())
        return torch.ones(lo, device="cuda"), big[:lo] if cc.data_ptr() == c.data_ptr() else big[-lo:]

    mos, d = fo.run(score, c, c, None, 2)
    assert d.dtype == torch.int32 and mos.dtype == torch.float32
    np.testing.assert_array_equal(d.cpu().numpy(), big.cpu().numpy())


def test_forced_copy_branch_on_one_gpu(pairs):
    """The peer-copy branch of a shard whose rows live on another device, run on
    the 1-GPU box by FanOut.force_copy: each shard's rows are copied on its own copy stream of the
    source device, after the event of the caller's stream, and its compute stream waits for the
    copy's event -- scores bitwise those of the single-device call, also from a non-default caller
    stream, and the recorded input streams are the per-shard copy streams, not the compute
    streams."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    want = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n))
    m = PESQ_STOI(16000, use_gpu=True, devices=[0, 0, 0])
    m._fanout.force_copy = True
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream())
        # inputs produced on the caller's stream right before the call: the copies must wait for them
        c2, n2 = c * 1.0, n * 1.0
        got = m.scores(c2, n2)
        res = m(c2, n2)
        got = [t.clone() for t in got]
    s.synchronize()
    for a, b in zip(_np(got), want):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(np.array([d["PESQ"] for d in res], np.float32), want[0])
    np.testing.assert_array_equal(np.array([d["ESTOI"] for d in res], np.float32), want[2])
    rec = m._fanout.last_copy_streams
    assert len(rec) == 3 and all(r is not None for r in rec)
    assert all(r["input"] != r["compute"] for r in rec)
    assert len({r["input"] for r in rec}) == 3
    assert s.cuda_stream not in {r["input"] for r in rec}
    dev0 = torch.device("cuda", 0)
    assert {r["input"] for r in rec} == {m._fanout._copy_stream(k, dev0).cuda_stream for k in range(3)}


def test_host_slots_keyed_by_device(pairs):
    """The drop-in call's pinned score buffer and event are kept per (thread, device)."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    m(c, n)
    assert set(m.__dict__["_fsem_tls"].slots) == {0}
    m.release()
    assert "_held_list" not in m.__dict__ and not m.__dict__["_fsem_tls"].slots
    assert [d["PESQ"] for d in m(c, n)] == [d["PESQ"] for d in PESQ_STOI(16000, use_gpu=True)(c, n)]


needs_two = pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two HIP devices")


@needs_two
def test_two_devices_peer_copies(pairs):
    """devices=[0, 1] with the batch on cuda:0: shard 1 pulls its rows over xGMI on its copy stream of
    cuda:0 and its scores come back to cuda:0; bitwise the single-device scores, from a non-default
    caller stream."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    want = _np(PESQ_STOI(16000, use_gpu=True).scores(c, n))
    m = PESQ_STOI(16000, use_gpu=True, devices=[0, 1])
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        s.wait_stream(torch.cuda.default_stream())
        got = [t.clone() for t in m.scores(c, n)]
    s.synchronize()
    assert all(t.device == torch.device("cuda", 0) for t in got)
    for a, b in zip(_np(got), want):
        np.testing.assert_array_equal(a, b)
    rec = m._fanout.last_copy_streams
    assert rec[0]["input"] == rec[0]["compute"]
    assert rec[1]["input"] == m._fanout._copy_stream(1, torch.device("cuda", 0)).cuda_stream != rec[1]["compute"]


@needs_two
def test_metric_called_on_two_devices(pairs):
    """One metric object called on cuda:0 and then with cuda:1 current: its per-thread
    host slot and event are per device, so the second call neither fails nor mixes devices."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n = pairs
    m = PESQ_STOI(16000, use_gpu=True)
    want = m(c, n)
    with torch.cuda.device(1):
        got = m(c.to("cuda:1"), n.to("cuda:1"))
    assert [d["PESQ"] for d in got] == [d["PESQ"] for d in want]
    assert [d["STOI"] for d in got] == [d["STOI"] for d in want]
    assert set(m.__dict__["_fsem_tls"].slots) == {0, 1}
