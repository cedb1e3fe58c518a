"""P.862-mode time alignment (P.862 sections 10.5-10.6 -- the histogram fine
stage and the recursive utterance split -- as restated in oracle/align_oracle.py steps 10-12 on
the fine stage's 320 ms pieces; PARITY UNPINNED against P.862 implementations, none is importable
here, and the reference has no time alignment, PESQ.py:19-22), CPU side: the oracle recovers known
per-utterance delays, an in-utterance delay change and two changes inside one utterance (which the
one-level utterance mode cannot); the package's CPU path gives the oracle's segments, delays and
aligned rows; PESQ(time_align="p862") scores the segment-aligned rows; the vote and split rules."""
import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, _cpu
from fast_speech_enhancement_metrics_amd.alignment import time_align, time_align_segments
from oracle import align_oracle as A

from tests import align_cases as AC


@pytest.fixture(scope="module")
def p862_batch():
    c, d = AC.batch()
    return c, d, A.align_p862(c, d)


def test_oracle_recovers_utterance_delays(p862_batch):
    _, _, (_, ds, segs) = p862_batch
    for (st, dl), case in zip(segs, AC.CASES):
        assert list(dl) == case[3]
        assert st[0] == 0 and st[-1] == AC.L_UTT and np.all(np.diff(st) > 0)
    assert abs(int(segs[1][0][1]) - 30000) <= A.CHUNK
    np.testing.assert_array_equal(ds, [int(dl[int(np.argmax(np.diff(st)))]) for st, dl in segs])


def test_two_levels_inside_one_utterance():
    c, d = AC.continuous_pair(3, AC.L_CONT, AC.CONT_PIECES)
    assert len(A.utterances(A.envelope(c.astype(np.float64)))) == 1
    st, dl, D = A.segments_p862(c, d)
    assert list(dl) == [100, 400, -200]
    for k, (a, _, _) in enumerate(AC.CONT_PIECES[1:], start=1):
        assert abs(int(st[k]) - a) <= A.CHUNK
    assert D == 400  # the longest segment's
    # the one-level utterance mode finds one change only
    assert len(A.segments(c, d)[1]) == 2


def test_cpu_path_matches_oracle(p862_batch):
    c, d, (out, ds, segs) = p862_batch
    al, dl, ns, st, sd = time_align_segments(torch.from_numpy(c), torch.from_numpy(d), mode="p862")
    np.testing.assert_array_equal(dl.numpy(), ds)
    for b, (s_o, d_o) in enumerate(segs):
        k = int(ns[b])
        np.testing.assert_array_equal(st[b, :k + 1].numpy(), s_o)
        np.testing.assert_array_equal(sd[b, :k].numpy(), d_o)
    np.testing.assert_array_equal(al.numpy(), out)
    c3, d3 = AC.continuous_pair(3, AC.L_CONT, AC.CONT_PIECES)
    st_o, dl_o, D_o = A.segments_p862(c3, d3)
    st_c, dl_c, D_c = _cpu.time_align_utt_row(c3, d3, 16000, "p862")
    np.testing.assert_array_equal(st_c, st_o)
    np.testing.assert_array_equal(dl_c, dl_o)
    assert D_c == D_o


def test_pesq_scores_the_aligned_rows(p862_batch):
    c, d, (out, _, _) = p862_batch
    m = PESQ(16000, use_gpu=False, time_align="p862")
    got = m.scores(torch.from_numpy(c), torch.from_numpy(d))
    want = _cpu.pesq(torch.from_numpy(c), torch.from_numpy(out.astype(np.float32)))
    np.testing.assert_array_equal(got.numpy(), want.numpy())
    a2, d2 = time_align(torch.from_numpy(c), torch.from_numpy(d), mode="p862")
    np.testing.assert_array_equal(a2.numpy(), out)
    with pytest.raises(ValueError):
        time_align_segments(torch.from_numpy(c), torch.from_numpy(d), mode="row")


def test_vote_and_split_rules():
    d0 = 0
    lag = lambda D: D - d0 + A.FINE  # noqa: E731
    # piece peaks: 6 pieces at +100, then 6 at +300; weak pieces do not vote
    P = np.zeros((12, 2 * A.FINE + 1))
    for i in range(6):
        P[i, lag(100)] = 10.0 + i
        P[6 + i, lag(300)] = 9.0 + i
    v, idx = A.piece_peaks(P)
    assert A.split_p862(v, idx, 0, 12, d0) == [(0, 100), (6, 300)]
    Pn = P.copy()
    Pn[3] = 0.0
    Pn[3, lag(-50)] = 0.3  # 0.3 < 5 % of 14: no vote
    v, idx = A.piece_peaks(Pn)
    assert idx[3] == -1 and A.split_p862(v, idx, 0, 12, d0) == [(0, 100), (6, 300)]
    # one outlier piece inside a constant-delay range never splits it (a half needs two votes)
    Po = np.zeros((8, 2 * A.FINE + 1))
    for i in range(8):
        Po[i, lag(100 if i != 5 else 250)] = 10.0
    v, idx = A.piece_peaks(Po)
    assert A.split_p862(v, idx, 0, 8, d0) == [(0, 100)]
    # the CPU path's rules agree
    for M in (P, Pn, Po):
        v, idx = A.piece_peaks(M)
        assert _cpu._ta_split_p862(v, idx, 0, M.shape[0], d0, 0) == A.split_p862(v, idx, 0, M.shape[0], d0)
    # the histogram: the triangle-smoothed maximum, confidence = its share of the votes
    H = np.zeros((4, 2 * A.FINE + 1))
    H[0, lag(10)] = H[1, lag(12)] = H[2, lag(10)] = 1.0
    v, idx = A.piece_peaks(H)
    D, conf, nv = A.hist_delay(v, idx, 0, 4, d0)
    assert (D, nv) == (10, 3) and abs(conf - (2 * 9 + 7) / (9 * 3)) < 1e-12
