"""Variable-length batches and non-native input rates.

Golden vectors (tests/golden/make_golden.py, the reference run in the build container):
  rate_8k     uniform 8 kHz batch: PESQ(sample_rate=8000) resamples 8 -> 16 kHz, STOI 8 -> 10 kHz
              (base.py:13,19-20);
  varlen_16k  ragged 16 kHz batch, each expected score = the reference on that unpadded
  varlen_8k   utterance alone (NaN where the reference rejects it as too short); rows keep the
              signal past their length, which the engine must ignore.
The CPU tests pin the oracle and the CPU mode; the gpu tests run the HIP engine through the
drop-in API (list-of-utterances form and padded-tensor + lengths form).
"""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle, ta
from tests.conftest import load_golden

VARLEN = ["varlen_16k", "varlen_8k"]
PESQ_TOL, STOI_TOL = 5e-3, 5e-4  # engine vs reference (test_gpu_parity.py)


def _oracle_row(g, b):
    n = int(g["lengths"][b])
    sr = int(g["sample_rate"])
    c, d = g["clean_f"][b:b + 1, :n], g["noisy_f"][b:b + 1, :n]
    c16 = ta.resample(c, sr, 16000) if sr != 16000 else c
    d16 = ta.resample(d, sr, 16000) if sr != 16000 else d
    try:
        p = float(pesq_oracle.pesq(c16, d16)[0])
    except (RuntimeError, ValueError, IndexError):
        p = float("nan")
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        s, e = stoi_oracle.stoi(c, d, sr)
    return p, float(s[0]), float(e[0])


def _close_with_nans(got, want, atol):
    got, want = np.asarray(got, dtype=np.float64), np.asarray(want, dtype=np.float64)
    assert np.array_equal(np.isnan(got), np.isnan(want)), (got, want)
    m = ~np.isnan(want)
    np.testing.assert_allclose(got[m], want[m], atol=atol, rtol=0)


# ------------------------------------------------------------------------------- oracle pin
@pytest.mark.parametrize("name", VARLEN)
def test_oracle_varlen_matches_reference(name):
    g = load_golden(name)
    rows = [_oracle_row(g, b) for b in range(len(g["lengths"]))]
    _close_with_nans([r[0] for r in rows], g["pesq"], 2e-3)
    _close_with_nans([r[1] for r in rows], g["stoi"], 1e-5)
    _close_with_nans([r[2] for r in rows], g["estoi"], 1e-5)


def test_oracle_8k_matches_reference():
    g = load_golden("rate_8k")
    c16, d16 = ta.resample(g["clean_f"], 8000, 16000), ta.resample(g["noisy_f"], 8000, 16000)
    np.testing.assert_allclose(pesq_oracle.pesq(c16, d16), g["pesq"], atol=2e-3, rtol=0)
    s, e = stoi_oracle.stoi(g["clean_f"], g["noisy_f"], 8000)
    np.testing.assert_allclose(s, g["stoi"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(e, g["estoi"], atol=1e-5, rtol=0)


def test_varlen_golden_has_short_rows():
    g = load_golden("varlen_16k")
    assert np.isnan(g["pesq"]).any() and np.isnan(g["stoi"]).any()  # the NaN contract is exercised
    assert (g["lengths"] < g["clean"].shape[1]).sum() >= 4


# ------------------------------------------------------------------------------- host logic
def test_pad_batch_and_lengths():
    from fast_speech_enhancement_metrics_amd.batching import as_lengths, pad_batch, resampled_lengths
    c = [torch.ones(5), torch.ones(9)]
    d = [torch.zeros(5), torch.zeros(9)]
    pc, pd, lens = pad_batch(c, d)
    assert pc.shape == (2, 12) and lens.tolist() == [5, 9] and lens.dtype == torch.int32
    assert pc[0, 5:].abs().sum() == 0 and pc[1, :9].sum() == 9
    with pytest.raises(Exception, match="same shape"):
        pad_batch([torch.ones(5)], [torch.ones(6)])
    with pytest.raises(ValueError):
        as_lengths([3, 13], 2, 12)
    assert resampled_lengths(torch.tensor([24000, 16667, 11111]), 8000, 16000).tolist() == [48000, 33334, 22222]
    assert resampled_lengths(torch.tensor([16001]), 16000, 10000).tolist() == [10001]


# ------------------------------------------------------------------------------- CPU mode
def test_cpu_mode_8k_matches_reference():
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    g = load_golden("rate_8k")
    c, d = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"])
    np.testing.assert_allclose([r["PESQ"] for r in PESQ(8000)(c, d)], g["pesq"], atol=2e-3, rtol=0)
    res = STOI(8000)(c, d)
    np.testing.assert_allclose([r["STOI"] for r in res], g["stoi"], atol=1e-4, rtol=0)
    np.testing.assert_allclose([r["ESTOI"] for r in res], g["estoi"], atol=1e-4, rtol=0)


@pytest.mark.parametrize("name", VARLEN)
def test_cpu_mode_varlen_matches_reference(name):
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    g = load_golden(name)
    sr = int(g["sample_rate"])
    c, d, lens = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]), g["lengths"]
    _close_with_nans([r["PESQ"] for r in PESQ(sr)(c, d, lengths=lens)], g["pesq"], 2e-3)
    cl = [c[b, :n] for b, n in enumerate(lens)]
    dl = [d[b, :n] for b, n in enumerate(lens)]
    res = STOI(sr)(cl, dl)
    _close_with_nans([r["STOI"] for r in res], g["stoi"], 1e-4)
    _close_with_nans([r["ESTOI"] for r in res], g["estoi"], 1e-4)


# ------------------------------------------------------------------------------- GPU engine
@pytest.mark.gpu
def test_gpu_8k_matches_reference():
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    g = load_golden("rate_8k")
    c, d = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"])
    np.testing.assert_allclose([r["PESQ"] for r in PESQ(8000, use_gpu=True)(c, d)], g["pesq"], atol=PESQ_TOL, rtol=0)
    res = STOI(8000, use_gpu=True)(c, d)
    np.testing.assert_allclose([r["STOI"] for r in res], g["stoi"], atol=STOI_TOL, rtol=0)
    np.testing.assert_allclose([r["ESTOI"] for r in res], g["estoi"], atol=STOI_TOL, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("name", VARLEN)
@pytest.mark.parametrize("form", ["lists", "lengths"])
def test_gpu_varlen_matches_reference(name, form):
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    g = load_golden(name)
    sr = int(g["sample_rate"])
    c, d, lens = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]), g["lengths"]
    if form == "lists":
        args = ([c[b, :n] for b, n in enumerate(lens)], [d[b, :n] for b, n in enumerate(lens)])
        kw = {}
    else:  # padded rows holding signal past each length: must be ignored
        args, kw = (c, d), {"lengths": torch.from_numpy(lens)}
    _close_with_nans([r["PESQ"] for r in PESQ(sr, use_gpu=True)(*args, **kw)], g["pesq"], PESQ_TOL)
    res = STOI(sr, use_gpu=True)(*args, **kw)
    _close_with_nans([r["STOI"] for r in res], g["stoi"], STOI_TOL)
    _close_with_nans([r["ESTOI"] for r in res], g["estoi"], STOI_TOL)


@pytest.mark.gpu
def test_gpu_full_lengths_equal_uniform():
    """lengths == capacity for every row gives bit-identical scores to the uniform call."""
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    g = load_golden("pesq_ragged")
    c = torch.from_numpy(g["clean_f"]).cuda()
    d = torch.from_numpy(g["noisy_f"]).cuda()
    lens = torch.full((c.shape[0],), c.shape[1], dtype=torch.int32)
    p = PESQ(16000, use_gpu=True)
    assert torch.equal(p.scores(c, d), p.scores(c, d, lengths=lens))
    s = STOI(16000, use_gpu=True)
    a, b = s.scores(c, d, 16000), s.scores(c, d, 16000, lengths=lens)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


@pytest.mark.gpu
def test_gpu_varlen_large_mixed_batch():
    """A ragged batch of 64 utterances (1-12 s at 16 kHz) against per-utterance uniform calls
    of the engine itself (shared kernels, per-row geometry)."""
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    rng = np.random.default_rng(3)
    lens = rng.integers(16000, 192000, size=64)
    lens[:4] = [192000, 16000, 16001, 40077]
    cap = int(lens.max())
    c, d, _ = speech_like_pairs(64, cap, 16000, seed=21, device="cuda")
    p, s = PESQ(16000, use_gpu=True), STOI(16000, use_gpu=True)
    mos = p.scores(c, d, lengths=torch.from_numpy(lens.astype(np.int32))).cpu().numpy()
    st, es = (t.cpu().numpy() for t in s.scores(c, d, 16000, lengths=torch.from_numpy(lens.astype(np.int32))))
    for b in range(0, 64, 7):
        n = int(lens[b])
        m1 = p.scores(c[b:b + 1, :n].contiguous(), d[b:b + 1, :n].contiguous()).item()
        s1, e1 = (t.item() for t in s.scores(c[b:b + 1, :n].contiguous(), d[b:b + 1, :n].contiguous(), 16000))
        assert abs(mos[b] - m1) < 1e-4, (b, mos[b], m1)
        assert abs(st[b] - s1) < 1e-5 and abs(es[b] - e1) < 1e-5, (b, st[b], s1)


# ------------------------------------------------------------------------------- joint entry
def test_joint_cpu_mode_matches_reference():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    g = load_golden("varlen_16k")
    c, d, lens = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]), g["lengths"]
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        res = PESQ_STOI(16000)(c, d, lengths=lens)
    assert [sorted(r) for r in res] == [["ESTOI", "PESQ", "STOI"]] * len(lens)
    _close_with_nans([r["PESQ"] for r in res], g["pesq"], 2e-3)
    _close_with_nans([r["STOI"] for r in res], g["stoi"], 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["pesq_ragged", "stoi_16k_10s", "varlen_16k"])
def test_gpu_joint_bitwise_equals_separate_calls(name):
    """fsem_pesq_stoi_f32 (one read of the inputs) == fsem_pesq_wb_f32 + fsem_stoi_f32, bitwise."""
    from fast_speech_enhancement_metrics_amd import PESQ, PESQ_STOI, STOI
    g = load_golden(name)
    c = torch.from_numpy(g["clean_f"]).cuda()
    d = torch.from_numpy(g["noisy_f"]).cuda()
    lens = torch.from_numpy(g["lengths"]) if "lengths" in g else None
    mos, s, e = PESQ_STOI(16000, use_gpu=True).scores(c, d, lens)
    mos1 = PESQ(16000, use_gpu=True).scores(c, d, lens)
    s1, e1 = STOI(16000, use_gpu=True).scores(c, d, 16000, lengths=lens)
    assert torch.equal(mos, mos1, ) or torch.allclose(mos, mos1, atol=0, rtol=0, equal_nan=True)
    assert torch.allclose(s, s1, atol=0, rtol=0, equal_nan=True)
    assert torch.allclose(e, e1, atol=0, rtol=0, equal_nan=True)
    if "pesq" in g and "lengths" in g:
        _close_with_nans(mos.cpu().numpy(), g["pesq"], PESQ_TOL)
        _close_with_nans(s.cpu().numpy(), g["stoi"], STOI_TOL)


@pytest.mark.gpu
def test_gpu_joint_api_list_of_dicts():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    g = load_golden("varlen_16k")
    lens = g["lengths"]
    cl = [torch.from_numpy(g["clean_f"][b, :n]) for b, n in enumerate(lens)]
    dl = [torch.from_numpy(g["noisy_f"][b, :n]) for b, n in enumerate(lens)]
    res = PESQ_STOI(16000, use_gpu=True)(cl, dl)
    _close_with_nans([r["PESQ"] for r in res], g["pesq"], PESQ_TOL)
    _close_with_nans([r["STOI"] for r in res], g["stoi"], STOI_TOL)
    _close_with_nans([r["ESTOI"] for r in res], g["estoi"], STOI_TOL)


@pytest.mark.gpu
def test_gpu_front_y10_resampler_and_front_unchanged():
    """fsem_pesq_front_y10_f32: the 10 kHz rows match the reference's resampler (golden x10),
    the clean rows' VAD quarter sums match a float64 evaluation on those rows, and bark / power
    are bitwise those of fsem_pesq_front_f32."""
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    g = load_golden("stoi_16k")
    dev = torch.device("cuda")
    c = torch.from_numpy(g["clean_f"]).to(dev)
    d = torch.from_numpy(g["noisy_f"]).to(dev)
    B, L = c.shape
    F = lib.fsem_pesq_frames(L)
    L10 = (5 * L + 7) // 8
    y_ld = (L10 + 63) // 64 * 64
    v_ld = (L10 // 64 + 1 + 63) // 64 * 64
    vad = torch.full((B, v_ld, 2), float("nan"), device=dev)
    outs = []
    for joint in (False, True):
        bark = torch.full((2 * B, 49, (F + 31) // 32 * 32), -1.0, device=dev)
        power = torch.empty(2 * B, device=dev)
        y10 = torch.full((2 * B, y_ld), float("nan"), device=dev)
        ws = _native.workspace(lib.fsem_pesq_front_workspace_bytes(B, L), dev)
        h = _native.stream_handle(dev)
        if joint:
            rc = lib.fsem_pesq_front_y10_f32(c.data_ptr(), d.data_ptr(), B, L, L, None, bark.data_ptr(),
                                             power.data_ptr(), y10.data_ptr(), y_ld, vad.data_ptr(), v_ld,
                                             ws.data_ptr(), ws.numel(), h)
        else:
            rc = lib.fsem_pesq_front_f32(c.data_ptr(), d.data_ptr(), B, L, L, None, bark.data_ptr(),
                                         power.data_ptr(), ws.data_ptr(), ws.numel(), h)
        _native.check(rc, "front")
        outs.append((bark, power, y10))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    y = outs[1][2].cpu().numpy()
    np.testing.assert_allclose(y[0::2, :L10], g["x10_clean"], atol=2e-6, rtol=0)
    assert np.isfinite(y[1::2, :L10]).all()
    # VAD quarter sums of every complete 64-sample block of the clean rows (fsem_vad.h)
    w = torch.hann_window(257).numpy()[1:].astype(np.float64)
    nq = L10 // 64
    blocks = y[0::2, :64 * nq].astype(np.float64).reshape(B, nq, 64)
    par = (np.arange(nq) & 1)[:, None] * 64 + np.arange(64)[None, :]
    want = np.stack([((w[par] * blocks) ** 2).sum(-1), ((w[128 + par] * blocks) ** 2).sum(-1)], -1)
    got = vad.cpu().numpy()[:, :nq]
    np.testing.assert_allclose(got, want, rtol=2e-5, atol=1e-30)
    assert lib.fsem_pesq_front_y10_f32(c.data_ptr(), d.data_ptr(), B, L, L, None, c.data_ptr(), c.data_ptr(),
                                       c.data_ptr(), L10 - 1, None, 0, c.data_ptr(), 1 << 30, None) == -1
    assert lib.fsem_pesq_front_y10_f32(c.data_ptr(), d.data_ptr(), B, L, L, None, c.data_ptr(), c.data_ptr(),
                                       c.data_ptr(), y_ld, c.data_ptr(), v_ld - 64, c.data_ptr(), 1 << 30,
                                       None) == -1


def test_joint_8k_cpu_mode_matches_reference():
    """PESQ_STOI(8000): PESQ via 8->16 kHz, STOI via 8->10 kHz directly, as the reference."""
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    g = load_golden("varlen_8k")
    lens = g["lengths"]
    cl = [torch.from_numpy(g["clean_f"][b, :n]) for b, n in enumerate(lens)]
    dl = [torch.from_numpy(g["noisy_f"][b, :n]) for b, n in enumerate(lens)]
    res = PESQ_STOI(8000)(cl, dl)
    _close_with_nans([r["PESQ"] for r in res], g["pesq"], 2e-3)
    _close_with_nans([r["STOI"] for r in res], g["stoi"], 1e-4)
    _close_with_nans([r["ESTOI"] for r in res], g["estoi"], 1e-4)


@pytest.mark.gpu
def test_gpu_joint_8k_matches_reference():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    g = load_golden("rate_8k")
    res = PESQ_STOI(8000, use_gpu=True)(torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]))
    np.testing.assert_allclose([r["PESQ"] for r in res], g["pesq"], atol=PESQ_TOL, rtol=0)
    np.testing.assert_allclose([r["STOI"] for r in res], g["stoi"], atol=STOI_TOL, rtol=0)
    np.testing.assert_allclose([r["ESTOI"] for r in res], g["estoi"], atol=STOI_TOL, rtol=0)
