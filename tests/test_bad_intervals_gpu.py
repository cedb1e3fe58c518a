"""P.862's realignment of bad intervals on the GPU (fsem_pesq_bad_intervals_f32 +
fsem_pesq_pool_f32, csrc/align.hip ta_bad_*) against the oracle (oracle/align_oracle.py steps
13-15; PARITY UNPINNED against P.862 implementations -- the reference has no time alignment,
PESQ.py:19-22): from the engine's own per-frame disturbances, the intervals, their delays and the
second rows are bitwise the oracle's; the intervals recover the known delay jumps of
tests/align_cases.py; the MOS is the float64 pooling of the engine's frames (1e-6) and the oracle's
whole chain within the PESQ bar (5e-3); rows without an interval score as plain PESQ of the
aligned rows; ragged rows as unpadded ones; argument checks."""
import ctypes

import numpy as np
import pytest
import torch

from fast_speech_enhancement_metrics_amd import PESQ, _native
from fast_speech_enhancement_metrics_amd.alignment import realign_bad_intervals, time_align_segments
from oracle import align_oracle as A
from oracle import pesq_oracle as po
from tests import align_cases as AC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def run(dev):
    c, d = AC.bad_batch()
    ct, dt = torch.from_numpy(c).to(dev), torch.from_numpy(d).to(dev)
    m = PESQ(16000, use_gpu=True, time_align="p862")
    out = m.p862_scores(ct, dt)
    aligned, _, nseg, st, sd = time_align_segments(ct, dt, mode="p862")
    ds, _, fr1 = m.frame_disturbances(ct, aligned)
    nb, bd, second = realign_bad_intervals(ct, dt, aligned, fr1, nseg, st, sd)
    _, _, fr2 = m.frame_disturbances(ct, second)
    torch.cuda.synchronize()
    return dict(c=c, d=d, ct=ct, dt=dt, m=m, out=out, aligned=aligned, nseg=nseg, st=st, sd=sd, ds=ds, fr1=fr1,
                nb=nb, bd=bd, second=second, fr2=fr2)


def _pool64(fr1, fr2, bad):
    """float64 MOS of [B, 2, F] frames, each interval taking fr2's frames when their symmetric sum is
    smaller (oracle step 15)."""
    s, a = fr1[:, 0].astype(np.float64), fr1[:, 1].astype(np.float64)
    for b, iv in enumerate(bad):
        for f0, f1, _ in iv:
            if fr2[b, 0, f0:f1].astype(np.float64).sum() < fr1[b, 0, f0:f1].astype(np.float64).sum():
                s[b, f0:f1] = fr2[b, 0, f0:f1]
                a[b, f0:f1] = fr2[b, 1, f0:f1]
    return po.mos_from_distances(po.overlapping_sums(s), po.overlapping_sums(a))


def test_intervals_and_second_rows_match_oracle(run):
    c, d = run["c"], run["d"]
    al = run["aligned"].cpu().numpy()
    s1 = run["fr1"][:, 0].cpu().numpy()
    nb, bd, sec = run["nb"].cpu().numpy(), run["bd"].cpu().numpy(), run["second"].cpu().numpy()
    st, sd, ns = run["st"].cpu().numpy(), run["sd"].cpu().numpy(), run["nseg"].cpu().numpy()
    for b in range(c.shape[0]):
        k = int(ns[b])
        res_o, sec_o = A.realign_bad(c[b], d[b], al[b], st[b, :k + 1], sd[b, :k], s1[b])
        assert int(nb[b]) == len(res_o)
        assert [tuple(x) for x in bd[b, :len(res_o)].tolist()] == res_o
        np.testing.assert_array_equal(sec[b], sec_o)
    # the scoring chain made the same intervals
    np.testing.assert_array_equal(run["out"][2].cpu().numpy(), nb)
    np.testing.assert_array_equal(run["out"][3].cpu().numpy(), bd)


def test_intervals_recover_the_jumps(run):
    nb, bd = run["nb"].cpu().numpy(), run["bd"].cpu().numpy()
    for b, (_, jumps, want) in enumerate(AC.BAD_CASES):
        iv = bd[b, :int(nb[b])].tolist()
        if want is not None:
            assert [D for _, _, D in iv] == want
        for f0, f1, _ in iv:
            assert any(A.HOP * f0 < e and A.HOP * f1 + A.HOP > s for s, e, _ in jumps)


def test_mos_is_the_pooling_of_the_engine_frames(run):
    fr1, fr2 = run["fr1"].cpu().numpy(), run["fr2"].cpu().numpy()
    nb, bd = run["nb"].cpu().numpy(), run["bd"].cpu().numpy()
    bad = [[tuple(x) for x in bd[b, :int(nb[b])].tolist()] for b in range(fr1.shape[0])]
    want = _pool64(fr1, fr2, bad)
    got = run["out"][0].cpu().numpy()
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-6)
    # the oracle's whole chain (its own alignment, frames, intervals): the PESQ bar
    mos_o, bad_o = A.pesq_p862(run["c"], run["d"])
    np.testing.assert_allclose(got, mos_o, rtol=0, atol=5e-3)
    # rows with an interval score higher than without the realignment
    plain = PESQ(16000, use_gpu=True).scores(run["ct"], run["aligned"]).cpu().numpy()
    for b in range(len(bad)):
        if bad[b]:
            assert got[b] > plain[b] + 0.05
        else:
            assert abs(got[b] - plain[b]) <= 1e-6


def test_scores_entry_and_ragged_rows(run, dev):
    m = run["m"]
    got = m.scores(run["ct"], run["dt"])
    torch.testing.assert_close(got, run["out"][0], rtol=0, atol=0)
    c, d = run["c"], run["d"]
    pad = 4000
    cp = torch.from_numpy(np.pad(c, ((0, 0), (0, pad)))).to(dev)
    dp = torch.from_numpy(np.pad(d, ((0, 0), (0, pad)))).to(dev)
    got2 = m.scores(cp, dp, lengths=[AC.L_UTT] * c.shape[0])
    torch.testing.assert_close(got2, got, rtol=0, atol=2e-6)
    # a short row (< 20 frames) and an empty one score NaN; the others as alone
    lens = [AC.L_UTT, 3000, 0, AC.L_UTT]
    got3 = m.scores(run["ct"], run["dt"], lengths=lens).cpu().numpy()
    assert np.isnan(got3[1]) and np.isnan(got3[2])
    np.testing.assert_allclose(got3[[0, 3]], got.cpu().numpy()[[0, 3]], rtol=0, atol=2e-6)


def test_argument_checks(run, dev):
    lib = _native.load()
    B, L = run["ct"].shape
    p = run["fr1"].data_ptr()
    mos = torch.empty(B, device=dev)
    assert lib.fsem_pesq_pool_f32(None, p, run["ds"].data_ptr(), B, L, None, run["nb"].data_ptr(),
                                  run["bd"].data_ptr(), mos.data_ptr(), None) == _native.FSEM_EINVAL
    assert lib.fsem_pesq_pool_f32(p, p, run["ds"].data_ptr(), B, 600, None, run["nb"].data_ptr(),
                                  run["bd"].data_ptr(), mos.data_ptr(), None) == _native.FSEM_ESHORT
    ws = lib.fsem_pesq_bad_intervals_workspace_bytes(B, L)
    assert ws > 0 and lib.fsem_pesq_bad_intervals_workspace_bytes(0, L) == 0
    buf = torch.empty(8, dtype=torch.uint8, device=dev)
    a = run["aligned"]
    r = lib.fsem_pesq_bad_intervals_f32(run["ct"].data_ptr(), run["dt"].data_ptr(), a.data_ptr(), B, L, L, None, p,
                                        run["nseg"].data_ptr(), run["st"].data_ptr(), run["sd"].data_ptr(),
                                        run["nb"].data_ptr(), run["bd"].data_ptr(), a.data_ptr(), a.stride(0),
                                        buf.data_ptr(), ctypes.c_size_t(8), None)
    assert r == _native.FSEM_EWORKSPACE
    with pytest.raises(ValueError):
        realign_bad_intervals(run["ct"], run["dt"], a, run["fr1"][:, :, :10], run["nseg"], run["st"], run["sd"])


def test_random_plans_against_cpu_path(dev):
    """Random plans at 10 s (1-3 jumps of 120-250 ms by 100-380 samples off the row's delay): the
    engine's intervals and delays equal the package's float64 CPU path on >= 80 % of the rows (a
    frame disturbance near the threshold of 30 can move an interval's edge between float32 and
    float64 models), and those rows' MOS within the PESQ bar."""
    from fast_speech_enhancement_metrics_amd import _cpu
    L = 160000
    rng = np.random.default_rng(41)
    rows = []
    for b in range(12):
        jumps, t = [], 8000
        for _ in range(int(rng.integers(1, 4))):
            t += int(rng.integers(6000, 30000))
            ln = int(rng.integers(2000, 4000))
            if t + ln > L - 8000:
                break
            jumps.append((t, t + ln, 150 + int(rng.choice([-1, 1])) * int(rng.integers(100, 380))))
            t += ln
        rows.append(AC.gated_pair(900 + b, L, jumps))
    c = np.stack([r[0] for r in rows])
    d = np.stack([r[1] for r in rows])
    g = PESQ(16000, use_gpu=True, time_align="p862").p862_scores(torch.from_numpy(c).to(dev),
                                                                 torch.from_numpy(d).to(dev))
    h = _cpu.pesq_p862(torch.from_numpy(c), torch.from_numpy(d))
    g = [t.cpu().numpy() for t in g]
    h = [t.numpy() for t in h]
    same, found = 0, 0
    for b in range(len(rows)):
        k = int(g[2][b])
        found += k > 0
        if k == int(h[2][b]) and np.array_equal(g[3][b, :k], h[3][b, :k]):
            same += 1
            assert abs(float(g[0][b]) - float(h[0][b])) <= 5e-3, (b, g[0][b], h[0][b])
    assert found >= len(rows) // 2, found
    assert same >= 0.8 * len(rows), same
