"""BASELINE.json configs at their stated per-GPU size, checked by size-independent properties
(sampled rows against the oracle -- the CPU restatement of the reference pinned by tests/golden --
batch independence, finiteness, ranges):

* configs[2]: STOI + ESTOI of 8192 x 5 s @ 16 kHz pairs on one GPU (fused 16 -> 10 kHz);
* configs[4]: one GPU's shard of the 16384-utterance mixed batch on 8 GPUs -- 2048 ragged rows,
  lengths uniform in 2-30 s, half at 8 kHz (PESQ via 8 -> 16 kHz, STOI via 8 -> 10 kHz, as the
  reference's PESQ(8000) / STOI(8000)) and half at 16 kHz (joint entry), per-row lengths; the
  rows of rank 0 under the LPT plan for 8 ranks (distributed.lpt_shards), as bench.py --workload c5.

Tolerances: PESQ 5e-3, STOI / ESTOI 5e-4 (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4


def test_config3_stoi_8192x5s():
    from fast_speech_enhancement_metrics_amd import STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    B, L = 8192, 80000
    cs, ns = [], []
    for lo in range(0, B, 2048):
        c, n, _ = speech_like_pairs(2048, L, 16000, seed=77 + lo, device="cuda")
        cs.append(c)
        ns.append(n)
    c, n = torch.cat(cs), torch.cat(ns)
    del cs, ns
    m = STOI(16000, use_gpu=True)
    s, e = (t.cpu().numpy() for t in m.scores(c, n, 16000))
    assert s.shape == (B,) and np.isfinite(s).all() and np.isfinite(e).all()
    assert (np.abs(s) <= 1).all() and (np.abs(e) <= 1).all()
    s2, e2 = (t.cpu().numpy() for t in m.scores(c, n, 16000))
    np.testing.assert_array_equal(s2, s)  # deterministic
    np.testing.assert_array_equal(e2, e)
    rows = [0, 1, 4095, 4096, 6553, 8191]  # 6553: the first row past 2^31 bytes per signal buffer
    idx = torch.tensor(rows, device="cuda")
    ss, se = (t.cpu().numpy() for t in m.scores(c[idx].contiguous(), n[idx].contiguous(), 16000))
    np.testing.assert_array_equal(ss, s[rows])  # STOI is batch-independent bitwise
    np.testing.assert_array_equal(se, e[rows])
    os_, oe = stoi_oracle.stoi(c[idx].cpu().numpy(), n[idx].cpu().numpy(), 16000)
    ds, de = np.abs(s[rows] - os_).max(), np.abs(e[rows] - oe).max()
    print(f"config 3 rows {rows}: max |dSTOI| {ds:.2e} |dESTOI| {de:.2e} vs oracle")
    assert ds < STOI_TOL and de < STOI_TOL


def _c5_shard(world=8, rank=0, per_gpu=2048):
    """bench.py --workload c5's plan: the rows rank `rank` scores."""
    from fast_speech_enhancement_metrics_amd.distributed import lpt_shards
    n_total = per_gpu * world
    rng = np.random.default_rng(5)
    secs = rng.uniform(2.0, 30.0, size=n_total)
    rate = np.where(np.arange(n_total) % 2 == 0, 8000, 16000)
    lens = np.round(secs * rate).astype(np.int64)
    cost = np.where(rate == 8000, 2 * lens, lens)
    mine = np.array(lpt_shards(cost, world)[rank], dtype=np.int64)
    return mine, rate, lens


def test_config5_shard_ragged_mixed_rates():
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    mine, rate, lens = _c5_shard()
    assert 1900 < len(mine) < 2200  # LPT by 16 kHz-equivalent length: ~2048 rows per rank
    checked = 0
    for sr in (8000, 16000):
        idx = mine[rate[mine] == sr]
        ln = lens[idx]
        cap = int(-(-int(ln.max()) // 4) * 4)
        cs, ns = [], []
        for lo in range(0, len(idx), 256):
            c, n, _ = speech_like_pairs(min(256, len(idx) - lo), cap, sr, seed=1000 + lo + sr, device="cuda")
            cs.append(c)
            ns.append(n)
        c, n = torch.cat(cs), torch.cat(ns)
        del cs, ns
        lt = torch.from_numpy(ln.astype(np.int32)).cuda()
        if sr == 16000:
            mos, s, e = (t.cpu().numpy() for t in PESQ_STOI(16000, use_gpu=True).scores(c, n, lengths=lt))
        else:
            mos = PESQ(8000, use_gpu=True).scores(c, n, lengths=lt, sample_rate=8000).cpu().numpy()
            s, e = (t.cpu().numpy() for t in STOI(8000, use_gpu=True).scores(c, n, 8000, lengths=lt))
        assert np.isfinite(mos).all() and np.isfinite(s).all() and np.isfinite(e).all(), sr  # every row >= 2 s
        assert (mos >= 1.0).all() and (mos <= 4.65).all() and (np.abs(s) <= 1).all()
        # sampled rows: shortest, longest, and two between -- each against the oracle on the
        # unpadded row alone (the row's result is the reference called on that row alone)
        order = np.argsort(ln)
        pick = [int(order[0]), int(order[len(order) // 3]), int(order[2 * len(order) // 3]), int(order[-1])]
        for r in pick:
            cr = c[r, :ln[r]].cpu().numpy()[None]
            nr = n[r, :ln[r]].cpu().numpy()[None]
            if sr == 16000:
                op = pesq_oracle.pesq(cr, nr)
            else:
                from oracle import ta
                op = pesq_oracle.pesq(ta.resample(cr, 8000, 16000), ta.resample(nr, 8000, 16000))
            os_, oe = stoi_oracle.stoi(cr, nr, sr)
            dp, ds, de = abs(mos[r] - op[0]), abs(s[r] - os_[0]), abs(e[r] - oe[0])
            print(f"config 5 shard {sr} Hz row {r} ({ln[r] / sr:.1f} s): |dPESQ| {dp:.2e} |dSTOI| {ds:.2e} "
                  f"|dESTOI| {de:.2e}")
            assert dp < PESQ_TOL and ds < STOI_TOL and de < STOI_TOL
            checked += 1
        # ragged equivalence: the picked rows scored as their own small padded batch
        pi = torch.tensor(pick, device="cuda")
        sub_l = lt[pi]
        if sr == 16000:
            m2, s2, e2 = (t.cpu().numpy() for t in
                          PESQ_STOI(16000, use_gpu=True).scores(c[pi].contiguous(), n[pi].contiguous(), lengths=sub_l))
        else:
            m2 = PESQ(8000, use_gpu=True).scores(c[pi].contiguous(), n[pi].contiguous(), lengths=sub_l,
                                                 sample_rate=8000).cpu().numpy()
            s2, e2 = (t.cpu().numpy() for t in STOI(8000, use_gpu=True).scores(c[pi].contiguous(), n[pi].contiguous(),
                                                                                8000, lengths=sub_l))
        np.testing.assert_allclose(m2, mos[pick], atol=1e-5, rtol=0)  # back-end wave form may differ
        np.testing.assert_array_equal(s2, s[pick])
        np.testing.assert_array_equal(e2, e[pick])
        del c, n
    assert checked == 8
