"""Utterance-mode time alignment (P.862 sections 10.3-10.5 as restated in
oracle/align_oracle.py steps 5-9 -- PARITY UNPINNED against P.862 implementations, none is
importable here, and the reference has no time alignment, PESQ.py:19-22), CPU side: the oracle
recovers known per-utterance delays and an in-utterance delay change (split) of synthetic pairs
(tests/align_cases.py); the package's CPU path (_cpu.time_align_utterances, FFT correlations)
gives the oracle's segments, delays and aligned rows; PESQ(time_align="utterance") scores the
segment-aligned rows."""
import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, _cpu
from fast_speech_enhancement_metrics_amd.alignment import time_align, time_align_segments
from oracle import align_oracle as A

from tests import align_cases as AC


@pytest.fixture(scope="module")
def utt_batch():
    c, d = AC.batch()
    return c, d, A.align_utterances(c, d)


def test_oracle_recovers_utterance_delays(utt_batch):
    _, _, (_, ds, segs) = utt_batch
    for (st, dl), case in zip(segs, AC.CASES):
        assert list(dl) == case[3]
        assert st[0] == 0 and st[-1] == AC.L_UTT and np.all(np.diff(st) > 0)
    # the split case: the change lies inside the second segment's first piece or at its start
    st1 = segs[1][0]
    assert abs(int(st1[1]) - 30000) <= A.CHUNK
    # the row delay: the longest segment's
    np.testing.assert_array_equal(ds, [int(dl[int(np.argmax(np.diff(st)))]) for st, dl in segs])


def test_utterance_rules():
    env = np.zeros(1000)
    env[10:40] = 1.0       # 30 frames: joined with the next run (gap 20 < JOIN)
    env[60:100] = 1.0      # -> utterance (10, 100)
    env[200:230] = 1.0     # 30 frames alone: shorter than MINUTT, dropped
    env[400:470] = 1.0     # utterance (400, 470)
    assert A.utterances(env) == [(10, 100), (400, 470)]
    assert _cpu._ta_utterances(env) == [(10, 100), (400, 470)]
    assert A.region_starts([(10, 100), (400, 470)], 64000) == [0, 64 * 250, 64000]
    many = np.zeros(40 * 120)
    for k in range(40):
        many[120 * k:120 * k + 60] = 1.0
    u = A.utterances(many)
    assert len(u) == A.MAXU and u[-1] == (120 * (A.MAXU - 1), 120 * 39 + 60)
    assert _cpu._ta_utterances(many) == u
    rng = np.random.default_rng(3)
    for _ in range(20):
        e = (rng.random(3000) < rng.uniform(0.05, 0.95)).astype(float)
        assert _cpu._ta_utterances(e) == A.utterances(e)


def test_cpu_path_matches_oracle(utt_batch):
    c, d, (out, ds, segs) = utt_batch
    al, dl, ns, st, sd = time_align_segments(torch.from_numpy(c), torch.from_numpy(d))
    np.testing.assert_array_equal(dl.numpy(), ds)
    for b, (s_o, d_o) in enumerate(segs):
        k = int(ns[b])
        np.testing.assert_array_equal(st[b, :k + 1].numpy(), s_o)
        np.testing.assert_array_equal(sd[b, :k].numpy(), d_o)
    np.testing.assert_array_equal(al.numpy(), out)
    al2, dl2 = time_align(torch.from_numpy(c), torch.from_numpy(d), mode="utterance")
    np.testing.assert_array_equal(al2.numpy(), out)
    np.testing.assert_array_equal(dl2.numpy(), ds)


def test_cpu_path_ragged_and_empty_rows(utt_batch):
    c, d, _ = utt_batch
    lens = [AC.L_UTT, 50000, 0, 700]
    out, ds, segs = A.align_utterances(c, d, lengths=lens)
    al, dl, ns, st, sd = time_align_segments(torch.from_numpy(c), torch.from_numpy(d), lengths=lens)
    np.testing.assert_array_equal(al.numpy(), out)
    np.testing.assert_array_equal(dl.numpy(), ds)
    for b, (s_o, d_o) in enumerate(segs):
        k = int(ns[b])
        np.testing.assert_array_equal(st[b, :k + 1].numpy(), s_o)
        np.testing.assert_array_equal(sd[b, :k].numpy(), d_o)
    assert int(ns[2]) == 1 and int(st[2, 1]) == 0 and int(dl[2]) == 0
    assert not al[2].any() and not al[3, 700:].any()


def test_pesq_time_align_utterance_mode(utt_batch):
    c, d, (out, ds, _) = utt_batch
    m = PESQ(16000, time_align="utterance")
    got = m.scores(torch.from_numpy(c), torch.from_numpy(d))
    want = PESQ(16000).scores(torch.from_numpy(c), torch.from_numpy(out))
    np.testing.assert_array_equal(got.numpy(), want.numpy())
    np.testing.assert_array_equal(m.last_delays.numpy(), ds)
    with pytest.raises(ValueError):
        PESQ(16000, time_align="frames")
    with pytest.raises(ValueError):
        time_align(torch.from_numpy(c), torch.from_numpy(d), mode="frames")
