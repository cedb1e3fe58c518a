"""P.862's realignment of bad intervals (P.862 section 10.7 as restated in oracle/align_oracle.py
steps 13-15; PARITY UNPINNED against P.862 implementations, none is importable here, and the
reference has no time alignment, PESQ.py:19-22), CPU side: the oracle finds the short delay jumps
of tests/align_cases.py's gated rows as bad intervals, recovers their delays and raises the rows'
MOS; the interval rules (threshold, joining, minimum length, cap); the package's CPU path gives the
oracle's intervals, second rows and scores; PESQ(time_align="p862") scores through it, padded rows
with lengths as unpadded ones."""
import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, _cpu
from oracle import align_oracle as A
from oracle import pesq_oracle as po

from tests import align_cases as AC


@pytest.fixture(scope="module")
def bad_case():
    c, d = AC.bad_batch()
    mos, bad = A.pesq_p862(c, d)
    return c, d, mos, bad


def test_oracle_finds_and_realigns_the_jumps(bad_case):
    c, d, mos, bad = bad_case
    for (_, jumps, want), iv in zip(AC.BAD_CASES, bad):
        if want is not None:
            assert [D for _, _, D in iv] == want
        for f0, f1, _ in iv:  # every interval lies over a jump
            assert any(A.HOP * f0 < e and A.HOP * f1 + A.HOP > s for s, e, _ in jumps)
    al, _, _ = A.align_p862(c, d)
    plain = po.pesq(c, al)
    for b, iv in enumerate(bad):
        if iv:
            assert mos[b] > plain[b] + 0.05, (b, mos[b], plain[b])
        else:
            assert mos[b] == pytest.approx(plain[b], abs=1e-12)


def test_interval_rules():
    s = np.zeros(100)
    s[10:13] = 40.0               # 3 frames: too short
    s[20:23] = s[26:28] = 40.0    # gap of 3 (< 4): one interval [20, 28)
    s[40:43] = s[47:50] = 40.0    # gap of 4: two runs of 3, both too short
    s[60:66] = 31.0
    s[66] = 30.0                  # not above the threshold
    s[95:100] = 45.0              # up to the row's end
    assert A.bad_intervals(s) == [(20, 28), (60, 66), (95, 100)]
    assert _cpu.bad_runs(s) == A.bad_intervals(s)
    many = np.tile([40.0] * 5 + [0.0] * 4, 30)
    assert len(A.bad_intervals(many)) == A.MAXBAD == 16
    assert A.bad_intervals(many)[-1] == (15 * 9, 15 * 9 + 5)
    assert A.bad_intervals(np.zeros(0)) == [] == _cpu.bad_runs(np.zeros(0))
    rng = np.random.default_rng(3)
    for _ in range(300):
        x = np.where(rng.random(int(rng.integers(1, 200))) < rng.random(), 40.0, 10.0)
        assert _cpu.bad_runs(x) == A.bad_intervals(x)


def test_cpu_path_matches_oracle(bad_case):
    c, d, mos, bad = bad_case
    m, ds, nb, bd = _cpu.pesq_p862(torch.from_numpy(c), torch.from_numpy(d))
    for b, iv in enumerate(bad):
        assert int(nb[b]) == len(iv)
        assert [tuple(x) for x in bd[b, :len(iv)].tolist()] == iv
    np.testing.assert_allclose(m.numpy(), mos, rtol=0, atol=2e-4)
    # the second rows, from the oracle's own frames
    al, _, segs = A.align_p862(c, d)
    i1 = {}
    po.disturbances(c, al, i1)
    for b in range(c.shape[0]):
        res_o, sec_o = A.realign_bad(c[b], d[b], al[b], segs[b][0], segs[b][1], i1["sym_frame"][b])
        res_c, sec_c = _cpu.realign_bad_row(c[b], d[b], al[b], segs[b][0], segs[b][1], i1["sym_frame"][b])
        assert res_c == res_o
        np.testing.assert_array_equal(sec_c, sec_o)


def test_pesq_p862_mode_scores(bad_case):
    c, d, mos, bad = bad_case
    m = PESQ(16000, use_gpu=False, time_align="p862")
    got = m.scores(torch.from_numpy(c), torch.from_numpy(d))
    want = _cpu.pesq_p862(torch.from_numpy(c), torch.from_numpy(d))[0]
    np.testing.assert_array_equal(got.numpy(), want.numpy())
    pad = 4000
    cp = np.pad(c, ((0, 0), (0, pad)))
    dp = np.pad(d, ((0, 0), (0, pad)))
    lens = [AC.L_UTT] * c.shape[0]
    got2 = m.scores(torch.from_numpy(cp), torch.from_numpy(dp), lengths=lens)
    np.testing.assert_allclose(got2.numpy(), got.numpy(), rtol=0, atol=1e-9)
