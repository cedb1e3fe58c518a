"""Opt-in time alignment, CPU side: the oracle (oracle/align_oracle.py, the
P.862-style restatement -- PARITY UNPINNED against P.862 implementations, none is importable
here, and the reference itself has no time alignment, PESQ.py:19-22) recovers known delays of
synthetic pairs; the package's CPU path (FFT correlations, _cpu.time_align) matches the oracle's
delays and aligned rows exactly; PESQ(time_align=True) scores the aligned rows."""
import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, _cpu
from fast_speech_enhancement_metrics_amd.alignment import time_align
from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
from oracle import align_oracle as A

B, L = 10, 48000


def delayed_pairs(seed=21, batch=B, length=L, span=3000):
    """(clean, degraded delayed by D, D): degraded[n] = noisy[n - D] inside the row, else 0."""
    c, n, _ = speech_like_pairs(batch, length, 16000, seed=seed)
    rng = np.random.default_rng(seed)
    D = rng.integers(-span, span + 1, batch)
    D[0], D[1] = 0, 7
    deg = np.stack([A.shift(n[b].numpy(), -int(D[b])) for b in range(batch)])
    return c, torch.from_numpy(deg), D


@pytest.fixture(scope="module")
def pairs():
    return delayed_pairs()


def test_oracle_recovers_known_delays(pairs):
    c, deg, D = pairs
    _, got = A.align(c.numpy(), deg.numpy())
    np.testing.assert_array_equal(got, D)


def test_oracle_shift_and_zero_rows():
    x = np.arange(10, dtype=np.float32)
    np.testing.assert_array_equal(A.shift(x, 3), [3, 4, 5, 6, 7, 8, 9, 0, 0, 0])
    np.testing.assert_array_equal(A.shift(x, -2), [0, 0, 0, 1, 2, 3, 4, 5, 6, 7])
    np.testing.assert_array_equal(A.shift(x, 20), np.zeros(10))
    z = np.zeros(4000, dtype=np.float32)
    assert A.delay(z, z) == 0  # nothing correlates positively: no shift
    assert A.delay(z[:50], z[:50]) == 0  # under one envelope frame


def test_cpu_path_matches_oracle(pairs):
    c, deg, D = pairs
    al, ds = time_align(c, deg)
    oal, ods = A.align(c.numpy(), deg.numpy())
    assert ds.dtype == torch.int32
    np.testing.assert_array_equal(ds.numpy(), ods)
    np.testing.assert_array_equal(al.numpy(), oal)


def test_cpu_path_ragged_rows(pairs):
    c, deg, D = pairs
    lens = np.array([L, 40000, 30001, L, 25000, L, 47999, 36000, L, 20000])
    al, ds = time_align(c, deg, lengths=lens)
    oal, ods = A.align(c.numpy(), deg.numpy(), lengths=lens)
    np.testing.assert_array_equal(ds.numpy(), ods)
    np.testing.assert_array_equal(al.numpy(), oal)
    for b in range(B):
        assert not al[b, lens[b]:].any()


def test_max_delay_bounds_the_crude_search(pairs):
    c, deg, D = pairs
    b = int(np.argmax(np.abs(D)))
    assert abs(D[b]) > 1000
    _, ds = time_align(c[b:b + 1], deg[b:b + 1], max_delay=64)
    # crude lag limited to one 4 ms frame: the fine search (+-383) cannot reach the true delay
    assert abs(int(ds[0])) <= 64 + A.FINE
    assert int(ds[0]) == A.delay(c[b].numpy(), deg[b].numpy(), max_delay=64)


def test_pesq_time_align_scores_the_aligned_rows(pairs):
    c, deg, D = pairs
    m = PESQ(16000, time_align=True)
    got = m.scores(c, deg)
    np.testing.assert_array_equal(m.last_delays.numpy(), D)
    aligned = torch.from_numpy(np.stack([A.shift(deg[b].numpy(), int(D[b])) for b in range(B)]))
    np.testing.assert_array_equal(got.numpy(), _cpu.pesq(c, aligned).numpy())
    # the drop-in call as well; and the default (reference) behaviour is unaligned
    res = m(c, deg)
    assert [r["PESQ"] for r in res] == got.tolist()
    plain = PESQ(16000).scores(c, deg)
    assert PESQ(16000).time_align is False
    # misaligned rows score lower unaligned (rows near the MOS floor within 0.01)
    assert (plain[2:] <= got[2:] + 0.01).all() and float((got[2:] - plain[2:]).mean()) > 0.1


def test_time_align_errors():
    c = torch.zeros(2, 1000)
    with pytest.raises(Exception):
        time_align(c, torch.zeros(2, 999))
    with pytest.raises(ValueError):
        time_align(c, c, max_delay=-1)
