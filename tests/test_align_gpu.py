"""Opt-in time alignment on the GPU (fsem_time_align_f32, csrc/align.hip) against the oracle
(oracle/align_oracle.py; PARITY UNPINNED against P.862 implementations -- the reference has no
time alignment, PESQ.py:19-22): delays equal to the oracle's and to the known synthetic delays,
aligned rows bitwise the oracle's shift of the input, ragged rows, and PESQ(time_align=True)
equal to the engine's PESQ of the aligned rows.  At 512 x 10 s: every known delay recovered."""
import time

import numpy as np
import pytest
import torch

from oracle import align_oracle as A

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def _delayed(batch, length, seed, span):
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(batch, length, 16000, seed=seed)
    rng = np.random.default_rng(seed)
    D = rng.integers(-span, span + 1, batch)
    D[0], D[1] = 0, -5
    deg = np.stack([A.shift(n[b].numpy(), -int(D[b])) for b in range(batch)])
    return c.numpy(), deg, D


def test_engine_matches_oracle(dev):
    from fast_speech_enhancement_metrics_amd.alignment import time_align
    c, deg, D = _delayed(16, 48000, 31, 3000)
    al, ds = time_align(torch.from_numpy(c).to(dev), torch.from_numpy(deg).to(dev))
    oal, ods = A.align(c, deg)
    np.testing.assert_array_equal(ods, D)
    np.testing.assert_array_equal(ds.cpu().numpy(), ods)
    np.testing.assert_array_equal(al.cpu().numpy(), oal)


def test_engine_ragged_and_odd_lengths(dev):
    from fast_speech_enhancement_metrics_amd.alignment import time_align
    c, deg, D = _delayed(8, 40001, 32, 2500)  # odd capacity: padded to a multiple of 4
    lens = np.array([40001, 30000, 25555, 40000, 12345, 39999, 20000, 33333], dtype=np.int32)
    al, ds = time_align(torch.from_numpy(c).to(dev), torch.from_numpy(deg).to(dev),
                        lengths=torch.from_numpy(lens).to(dev))
    oal, ods = A.align(c, deg, lengths=lens)
    np.testing.assert_array_equal(ds.cpu().numpy(), ods)
    np.testing.assert_array_equal(al.cpu().numpy(), oal)


def test_engine_edge_rows(dev):
    from fast_speech_enhancement_metrics_amd.alignment import time_align
    z = torch.zeros(3, 4096, device=dev)
    al, ds = time_align(z, z)
    assert (ds == 0).all() and not al.any()
    x = torch.randn(2, 100, device=dev)  # one envelope frame: crude 0, fine search only
    _, ds = time_align(x, x)
    assert ds.tolist() == [A.delay(r, r) for r in x.cpu().numpy()] == [0, 0]


def test_engine_unbounded_max_delay(dev):
    """max_delay = 2**31 - 1 (the C-ABI's int32 maximum, alignment.py's clamp): the crude search
    covers every lag, as the CPU path and the oracle do (its frame count used to wrap in 32 bits,
    which turned the crude search off on the GPU)."""
    from fast_speech_enhancement_metrics_amd.alignment import time_align
    c, deg, D = _delayed(6, 48000, 36, 3000)
    big = 2**31 - 1
    _, ds = time_align(torch.from_numpy(c).to(dev), torch.from_numpy(deg).to(dev), max_delay=big)
    _, dcpu = time_align(torch.from_numpy(c), torch.from_numpy(deg), max_delay=big)
    np.testing.assert_array_equal(ds.cpu().numpy(), dcpu.numpy())
    np.testing.assert_array_equal(ds.cpu().numpy(), D)


def test_pesq_time_align_on_gpu(dev):
    from fast_speech_enhancement_metrics_amd import PESQ
    c, deg, D = _delayed(12, 48000, 33, 3000)
    ct, dt = torch.from_numpy(c).to(dev), torch.from_numpy(deg).to(dev)
    m = PESQ(16000, use_gpu=True, time_align=True)
    got = m.scores(ct, dt)
    np.testing.assert_array_equal(m.last_delays.cpu().numpy(), D)
    aligned = torch.from_numpy(np.stack([A.shift(deg[b], int(D[b])) for b in range(12)])).to(dev)
    np.testing.assert_array_equal(got.cpu().numpy(), PESQ(16000, use_gpu=True).scores(ct, aligned).cpu().numpy())
    assert [r["PESQ"] for r in m(ct, dt)] == got.cpu().tolist()


def test_bench_size_recovers_every_delay(dev):
    """512 x 10 s with delays in +-2000 samples: every delay found; 4 rows against the oracle."""
    from fast_speech_enhancement_metrics_amd.alignment import time_align
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    Bn, Ln = 512, 160000
    c, n, _ = speech_like_pairs(Bn, Ln, 16000, seed=34, device=dev)
    rng = np.random.default_rng(34)
    D = torch.from_numpy(rng.integers(-2000, 2001, Bn)).to(dev)
    t = torch.arange(Ln, device=dev)
    src = t[None, :] - D[:, None]
    deg = torch.where((src >= 0) & (src < Ln), n.gather(1, src.clamp(0, Ln - 1)), torch.zeros_like(n))
    time_align(c, deg)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    al, ds = time_align(c, deg)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    print(f"time_align {Bn} x {Ln}: {ms:.2f} ms ({ms / Bn * 4096:.1f} ms per 4096 rows)")
    assert (ds.long() == D).all(), int((ds.long() != D).sum())
    for b in (0, 1, 200, 511):
        assert int(ds[b]) == A.delay(c[b].cpu().numpy(), deg[b].cpu().numpy())


def test_pesq_time_align_ragged_rows(dev):
    """PESQ(time_align=True) with per-row lengths: each row aligned within its own length, then
    scored as that row alone (the engine's PESQ of the oracle-aligned rows, bitwise)."""
    from fast_speech_enhancement_metrics_amd import PESQ
    c, deg, D = _delayed(6, 48000, 35, 2000)
    lens = np.array([48000, 40000, 36001, 47999, 30000, 44444], dtype=np.int32)
    ct, dt = torch.from_numpy(c).to(dev), torch.from_numpy(deg).to(dev)
    lt = torch.from_numpy(lens).to(dev)
    m = PESQ(16000, use_gpu=True, time_align=True)
    got = m.scores(ct, dt, lengths=lt).cpu().numpy()
    oal, ods = A.align(c, deg, lengths=lens)
    np.testing.assert_array_equal(m.last_delays.cpu().numpy(), ods)
    want = PESQ(16000, use_gpu=True).scores(ct, torch.from_numpy(oal).to(dev), lengths=lt).cpu().numpy()
    np.testing.assert_array_equal(got, want)
