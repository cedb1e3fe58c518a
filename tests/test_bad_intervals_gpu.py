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


def test_operands_checked_and_moved(run):
    """Operand shapes are checked before any launch (a short segment table would be read past its
    end on the GPU); operands held on the host are moved to the rows' device, same results."""
    ct, dt, a = run["ct"], run["dt"], run["aligned"]
    fr1, nseg, st, sd = run["fr1"], run["nseg"], run["st"], run["sd"]
    for args in ((a, fr1, nseg, st[:, :10], sd), (a, fr1, nseg, st, sd[:, :10]), (a, fr1, nseg[:1], st, sd),
                 (a[:, :100], fr1, nseg, st, sd)):
        with pytest.raises(ValueError):
            realign_bad_intervals(ct, dt, *args)
    with pytest.raises(ValueError):
        realign_bad_intervals(ct, dt, a, fr1, torch.full_like(nseg, _native.ALIGN_MAX_SEGMENTS + 1), st, sd)
    nb, bd, second = realign_bad_intervals(ct, dt, a.cpu(), fr1.cpu(), nseg.cpu(), st.cpu(), sd.cpu())
    assert nb.device == ct.device and second.device == ct.device
    assert torch.equal(nb, run["nb"]) and torch.equal(bd, run["bd"]) and torch.equal(second, run["second"])


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


def test_interval_rules_on_synthetic_frames(dev):
    """ta_bad_find / ta_bad_pool on synthetic per-frame disturbances through the C-ABI: the
    oracle's interval rules bitwise (threshold, joining, minimum length, the cap of 16, runs up
    to the row's last frame, rows of fewer than 20 frames and empty rows without intervals), and
    the pooled MOS of mixed first / second frames against the float64 pooling."""
    lib = _native.load()
    L = 96000
    F = lib.fsem_pesq_frames(L)
    rng = np.random.default_rng(5)
    B = 6
    sym = rng.uniform(0.0, 25.0, (B, F)).astype(np.float32)
    sym[0, 100:103] = 40.0                    # too short
    sym[0, 200:203] = sym[0, 206:209] = 44.0  # joined across a gap of 3
    sym[1, :] = np.tile(np.r_[np.full(5, 45.0), np.full(4, 10.0)], F // 9 + 1)[:F]  # > 16 runs: cap
    sym[2, F - 6:] = 45.0                     # up to the last frame
    sym[3, 10:30] = 31.0                      # a row of 3000 samples (< 20 frames): none
    sym[4, 50:60] = 30.0                      # not above the threshold
    lens = np.array([L, L, L, 3000, L, 0], dtype=np.int32)
    frames = np.zeros((B, 2, F), np.float32)
    frames[:, 0] = sym
    frames[:, 1] = rng.uniform(0.0, 20.0, (B, F))
    frames2 = frames.copy()
    frames2[:, :, :] *= 0.5                   # the second scoring disturbs less everywhere
    c = torch.from_numpy(rng.standard_normal((B, L)).astype(np.float32)).to(dev)
    d = torch.roll(c, 40, dims=1).contiguous()
    fr = torch.from_numpy(frames).to(dev)
    i32 = dict(dtype=torch.int32, device=dev)
    nseg = torch.ones(B, **i32)
    st = torch.zeros(B, 33, **i32)
    st[:, 1] = torch.from_numpy(lens).to(dev)
    sd = torch.full((B, 32), 40, **i32)
    n_bad = torch.empty(B, **i32)
    bad = torch.zeros(B, 16, 3, **i32)
    second = torch.empty(B, L, device=dev)
    lt = torch.from_numpy(lens).to(dev)
    ws = torch.empty(lib.fsem_pesq_bad_intervals_workspace_bytes(B, L), dtype=torch.uint8, device=dev)
    assert lib.fsem_pesq_bad_intervals_f32(c.data_ptr(), d.data_ptr(), d.data_ptr(), B, L, L, lt.data_ptr(),
                                           fr.data_ptr(), nseg.data_ptr(), st.data_ptr(), sd.data_ptr(),
                                           n_bad.data_ptr(), bad.data_ptr(), second.data_ptr(), L, ws.data_ptr(),
                                           ws.numel(), None) == 0
    torch.cuda.synchronize()
    nb, bd = n_bad.cpu().numpy(), bad.cpu().numpy()
    want = []
    for b in range(B):
        Fb = lib.fsem_pesq_frames(int(lens[b]))
        iv = A.bad_intervals(sym[b, :Fb]) if Fb >= 20 else []
        want.append(iv)
        assert int(nb[b]) == len(iv), (b, nb[b], iv)
        assert [tuple(x[:2]) for x in bd[b, :len(iv)].tolist()] == iv
    assert want[0] == [(200, 209)] and len(want[1]) == 16 and want[2] == [(F - 6, F)] and want[3] == [] == want[4]
    # every interval's delay: the roll by 40 samples, found within +-383 of the segment's 40
    for b in range(B):
        for f0, f1, D in bd[b, :int(nb[b])].tolist():
            assert D == 40, (b, f0, f1, D)
    # pooling: interval frames from the second scoring, the rest from the first
    dist = torch.zeros(2, B, device=dev)
    dist[:, 5] = float("nan")
    mos = torch.empty(B, device=dev)
    fr2 = torch.from_numpy(frames2).to(dev)
    assert lib.fsem_pesq_pool_f32(fr.data_ptr(), fr2.data_ptr(), dist.data_ptr(), B, L, lt.data_ptr(),
                                  n_bad.data_ptr(), bad.data_ptr(), mos.data_ptr(), None) == 0
    got = mos.cpu().numpy()
    for b in range(B):
        Fb = lib.fsem_pesq_frames(int(lens[b]))
        if Fb < 20 or b == 5:
            assert np.isnan(got[b])
            continue
        s, a = frames[b, 0, :Fb].astype(np.float64), frames[b, 1, :Fb].astype(np.float64)
        for f0, f1 in want[b]:
            s[f0:f1] = frames2[b, 0, f0:f1]
            a[f0:f1] = frames2[b, 1, f0:f1]
        ref = po.mos_from_distances(po.overlapping_sums(s[None]), po.overlapping_sums(a[None]))[0]
        assert abs(got[b] - ref) <= 1e-6, (b, got[b], ref)


def test_wb_frames_entry_matches_stage_entries(run, dev):
    """fsem_pesq_wb_frames_f32 (the whole-metric path with the back end's intermediates, which the
    P.862 chain scores with): its scores are fsem_pesq_wb_f32's, and its distances and per-frame
    disturbances those of the stage entries (fsem_pesq_front_f32 + fsem_pesq_distances_f32 on
    unit-scaled rows) -- also for rows scaled by 1e-6 and 1e6, which the whole-metric path takes
    as they are."""
    from fast_speech_enhancement_metrics_amd.PESQ import _wb_frames
    lib = _native.load()
    m = PESQ(16000, use_gpu=True)
    ct, al = run["ct"], run["aligned"].contiguous()
    for sc in (1.0, 1e-6, 1e6):
        c, a = ct * sc, al * sc
        ds, fr = _wb_frames(lib, c, a, None)
        ds2, _, fr2 = m.frame_disturbances(c, a)
        torch.testing.assert_close(fr, fr2, rtol=2e-6, atol=0)
        torch.testing.assert_close(ds, ds2, rtol=2e-6, atol=0)
        B, L = c.shape
        mos = torch.empty(B, device=dev)
        dist = torch.empty(2, B, device=dev)
        frames = torch.empty(B, 2, lib.fsem_pesq_frames(L), device=dev)
        ws = _native.workspace(lib.fsem_pesq_workspace_bytes(B, L), dev)
        assert lib.fsem_pesq_wb_frames_f32(c.data_ptr(), a.data_ptr(), B, L, L, None, mos.data_ptr(),
                                           dist.data_ptr(), frames.data_ptr(), ws.data_ptr(), ws.numel(),
                                           None) == 0
        torch.testing.assert_close(mos, m.scores(c, a), rtol=0, atol=0)
    assert lib.fsem_pesq_wb_frames_f32(ct.data_ptr(), al.data_ptr(), 4, AC.L_UTT, AC.L_UTT, None, None, None,
                                       None, None, 0, None) == _native.FSEM_EINVAL
