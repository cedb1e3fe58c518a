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
    """8 kHz rows (PESQ 8->16 kHz, STOI 8->10 kHz per shard) and PESQ(time_align=True): delays
    and scores reassembled in row order."""
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
    a1 = PESQ(16000, use_gpu=True, time_align=True)
    want = a1.scores(c, deg).cpu().numpy()
    a2 = PESQ(16000, use_gpu=True, time_align=True, devices=[0, 0])
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
