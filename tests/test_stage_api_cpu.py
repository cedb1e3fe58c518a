"""The reference's stage surface (PESQ.py:63-230, STOI.py:26-198, utils/bark.py, utils/loudness.py)
on the drop-in import paths, CPU mode, against the reference's golden intermediates:
Bark bands (``bark``), symmetric / asymmetric distances (``sym`` / ``asym``), kept VAD frames
(``kept``), 1/3-octave envelopes (``tob``) and the 16 -> 10 kHz signal (``x10_clean``).

Tolerances: Bark bands 5e-3 relative to the row's peak band power (the reference's float32
order-10 IIR noise), distances 1e-4 relative (MOS = 4.5 - 0.1 sym - 0.0309
asym: <= 5e-4 in MOS, inside the PESQ bar), envelopes 1e-4 relative, kept counts exact.
"""
import warnings

import numpy as np
import pytest
import torch

from tests.conftest import load_golden


def test_module_paths_are_importable():
    import fast_se_metrics
    import fast_se_metrics.PESQ  # noqa: F401  (the reference's own modules import these paths)
    import fast_se_metrics.STOI  # noqa: F401
    import fast_se_metrics.utils.bark as bark
    import fast_se_metrics.utils.loudness as loud
    from fast_se_metrics.base import BaseMetric
    from fast_se_metrics.PESQ import PESQ
    from fast_se_metrics.STOI import STOI
    assert fast_se_metrics.PESQ is PESQ and fast_se_metrics.STOI is STOI  # as the reference's __init__
    assert issubclass(PESQ, BaseMetric) and issubclass(STOI, BaseMetric)
    assert len(bark.nr_of_hz_bands_per_bark_band_16k) == 49 and sum(bark.nr_of_hz_bands_per_bark_band_16k) == 256
    assert bark.Sp_16k == pytest.approx(6.910853e-6) and loud.Sl_16k == pytest.approx(0.1866055)
    assert loud.zwicker_power == 0.23 and len(loud.abs_thresh_power_16k) == 49


def test_reference_method_names_exist():
    from fast_se_metrics import PESQ, STOI
    p, s = PESQ(16000), STOI(10000)
    for name in ("align_level", "pre_emphasize", "equalize_ranges", "get_bark_bands", "equalize_bark_bands",
                 "get_overlapping_sums", "get_disturbances", "compute_metric", "prepare_audio", "prepare_inputs"):
        assert callable(getattr(p, name)), name
    for name in ("to_spec", "filter_bank", "loudness", "power_filter", "pre_filter", "taper_weights", "device",
                 "sample_rate", "resampler"):
        assert getattr(p, name) is not None, name
    for name in ("get_octave_band_matrix", "stft", "overlap_and_add", "remove_silent_frames", "normalize",
                 "compute_segments", "equalize_clip", "compute_correlation", "compute_stoi", "compute_metric"):
        assert callable(getattr(s, name)), name
    for name in ("octave_band_matrix", "window", "sampling_frequency", "win_length", "hop_length", "n_fft",
                 "num_octave_bands", "min_frequency", "N", "beta", "dynamic_range"):
        assert getattr(s, name) is not None, name


def test_interp_and_filterbank():
    from fast_se_metrics.utils.bark import BarkFilterBank, interp, width_of_band_bark_16k
    t = interp(width_of_band_bark_16k, 49)
    assert t.dtype == torch.float64 and np.allclose(t.numpy(), width_of_band_bark_16k)
    with pytest.raises(ValueError):
        interp(width_of_band_bark_16k, 50)  # beyond the table, as scipy's interp1d
    fb = BarkFilterBank(256, 49)
    assert fb.fbank.shape == (49, 256) and torch.equal(fb.fbank.sum(0), torch.ones(256))
    assert fb.fbank[0, 0] == 1 and fb.fbank[48, 236:].sum() == 20
    assert float(fb.total_width) == pytest.approx(sum(width_of_band_bark_16k[1:]))
    small = BarkFilterBank(128, 24)  # the generic construction (bands around each centre)
    assert small.fbank.shape == (24, 128) and (small.fbank.sum(0) <= 1).all()
    x = torch.rand(2, 3, 257, dtype=torch.float64)
    out = fb(x)
    assert out.dtype == torch.float64 and out.shape == (2, 3, 49)
    ref = torch.einsum("ij,klj->kli", fb.fbank.double(), x[:, :, :-1]) * fb.pow_dens_correction
    assert torch.allclose(out, ref)
    d = torch.randn(2, 3, 49, dtype=torch.float64)
    w = fb.width_bark
    want2 = fb.total_width * ((w * d / fb.total_width ** 0.5)[:, :, 1:] ** 2).sum(2).sqrt()
    assert torch.allclose(fb.weighted_norm(d, p=2), want2)
    want1 = fb.total_width * (w * d / fb.total_width)[:, :, 1:].abs().sum(2)
    assert torch.allclose(fb.weighted_norm(d, p=1), want1)


def test_loudness_model():
    from fast_se_metrics.utils.loudness import Loudness, abs_thresh_power_16k
    lo = Loudness(49)
    thr = torch.tensor(abs_thresh_power_16k, dtype=torch.float64)
    p = thr * torch.tensor([0.5] * 10 + [2.0] * 39, dtype=torch.float64)
    out = lo.loudness(p.reshape(1, 1, 49))[0, 0]
    assert (out[:10] == 0).all() and (out[10:] > 0).all()
    bands = torch.rand(2, 5, 49, dtype=torch.float64) * 1e6
    afp = lo.audible_frame_power(bands, 1.0)
    assert afp.shape == (2, 5, 1)
    assert torch.allclose(afp[..., 0], (bands * (bands > thr)).sum(2))
    silent = torch.zeros(2, 5, 1, dtype=torch.bool)
    silent[:, 0] = True
    m = lo.mean_audible_band_power(bands, silent)
    keep = (bands > thr * 100) & ~silent
    assert torch.allclose(m, (bands * keep).sum(1) / 5)


@pytest.mark.parametrize("name", ["pesq_3s", "pesq_ragged"])
def test_pesq_stages_match_reference(name):
    from fast_se_metrics import PESQ
    g = load_golden(name)
    c, n = torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"])
    m = PESQ(16000)
    ce, ne = m.equalize_ranges(c, n)
    speech = torch.cat([ce, ne], 0)
    bark = m.get_bark_bands(speech.clone())
    ref = g["bark"].astype(np.float64)
    assert bark.shape == ref.shape and bark.dtype == torch.float64
    rel = (np.abs(bark.numpy() - ref).max(axis=(1, 2)) / np.abs(ref).max(axis=(1, 2))).max()
    assert rel < 5e-3, rel
    # the level-alignment factor (PESQ.py:100) vs the golden's
    aligned = m.align_level(speech.clone())
    scale = (aligned.double() * speech.double()).sum(1) / speech.double().square().sum(1)
    np.testing.assert_allclose(scale.numpy(), g["level_scale"], rtol=3e-3)
    # pre-emphasis: taper in place, then the IIR -- spectrum + filterbank of it give the bands
    pre = m.pre_emphasize(aligned.clone())
    # the reference's stage dtypes: align_level / pre_emphasize float32 (lfilter keeps the input's),
    # get_bark_bands float64 (bark.py:204's float64 correction)
    assert aligned.dtype == torch.float32 and pre.dtype == torch.float32
    spec = m.to_spec(torch.nn.functional.pad(pre, (0, pre.shape[1] % 256))).swapaxes(1, 2)
    spec[:, :, 0] = 0.0
    bark2 = m.filter_bank(spec.double())
    np.testing.assert_allclose(bark2.numpy(), bark.numpy(), rtol=1e-3, atol=1e-6 * np.abs(ref).max())
    # back end stages -> the golden distances
    B = c.shape[0]
    ec, en = m.equalize_bark_bands(bark[:B], bark[B:])
    assert ec.shape == en.shape == bark[:B].shape
    sym, asym = m.get_disturbances(c, n)
    np.testing.assert_allclose(sym.numpy(), g["sym"], atol=1e-5, rtol=1e-4)
    np.testing.assert_allclose(asym.numpy(), g["asym"], atol=1e-5, rtol=1e-4)
    d = torch.rand(B, bark.shape[1], dtype=torch.float64)
    want = (d.unfold(1, 20, 10) ** 6).mean(2) ** (1 / 6)
    assert torch.allclose(m.get_overlapping_sums(d), (want ** 2).mean(1).sqrt())
    mos = 0.999 + 4 / (1 + torch.exp(-1.3669 * (4.5 - 0.1 * sym - 0.0309 * asym) + 3.8224))
    np.testing.assert_allclose(mos.numpy(), g["pesq"], atol=5e-3, rtol=0)


def test_stoi_stages_match_reference():
    from fast_se_metrics import STOI
    g = load_golden("stoi_16k")
    m = STOI(16000)
    c10, n10 = m.prepare_inputs(torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]))
    np.testing.assert_allclose(c10.numpy(), g["x10_clean"], atol=2e-6, rtol=0)
    cs, ns, lens = m.remove_silent_frames(c10, n10)
    kept = (lens // m.hop_length - 1).numpy()
    assert kept.tolist() == g["kept"].tolist()
    assert cs.shape == ns.shape == (c10.shape[0], int(lens.max()))
    segs = m.compute_segments(torch.cat([cs, ns], 0), torch.cat([lens, lens], 0))
    tob = torch.cat([segs[0], torch.stack([s[:, :, -1] for s in segs[1:]], 2)], 2).numpy()  # undo the windows
    B = c10.shape[0]
    for b in range(B):
        T = int(g["kept"][b]) - 2
        for sig in (b, B + b):
            ref = g["tob"][sig][:, :T]
            assert np.abs(tob[sig][:, :T] - ref).max() / np.abs(ref).max() < 1e-4
    # segment statistics through the reference's stage sequence (STOI.py:167-198)
    st = torch.stack(segs, 1)
    x, y = st[:B], st[B:]
    yc = m.equalize_clip(x, y)
    bound = x * (1 + 10 ** (15 / 20))
    assert (yc <= bound + 1e-6).all()
    xs, ys = m.normalize(x.clone(), 3), m.normalize(yc, 3)
    xe = m.normalize(m.normalize(x.clone(), 3), 2)
    ye = m.normalize(m.normalize(y.clone(), 3), 2)
    nseg = torch.clamp((lens - 512) // 128 - 30 + 2, min=0)
    mask = (torch.arange(st.shape[1])[None, :] < nseg[:, None]).to(x.dtype)
    s = m.compute_correlation(xs, ys, mask, extended=False) / nseg
    e = m.compute_correlation(xe, ye, mask, extended=True) / nseg
    np.testing.assert_allclose(s.numpy(), g["stoi"], atol=5e-4, rtol=0)
    np.testing.assert_allclose(e.numpy(), g["estoi"], atol=5e-4, rtol=0)
    s2, e2 = m.compute_stoi(c10, n10)
    np.testing.assert_allclose(s2.numpy(), g["stoi"], atol=5e-4, rtol=0)
    np.testing.assert_allclose(e2.numpy(), g["estoi"], atol=5e-4, rtol=0)


def test_overlap_and_add_vectorised():
    """Kept frames of utterances with 3, 0 and 2 frames: frame j of utterance b at 128 j."""
    from fast_se_metrics import STOI
    m = STOI(10000)
    frames = torch.randn(5, 256, dtype=torch.float64)
    lens = torch.tensor([3, 0, 2])
    sig, out_len = m.overlap_and_add(frames, lens)
    assert out_len.tolist() == [512, 128, 384] and sig.shape == (3, 512)
    want = torch.zeros(3, 512, dtype=torch.float64)
    k = 0
    for b, n in enumerate(lens.tolist()):
        for j in range(n):
            want[b, 128 * j:128 * j + 256] += frames[k]
            k += 1
    assert torch.allclose(sig, want)


def test_compute_stoi_too_short_warns():
    from fast_se_metrics import STOI
    m = STOI(10000)
    x = torch.randn(2, 3000)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        s, e = m.compute_stoi(x, x)
    assert any(issubclass(i.category, RuntimeWarning) for i in w)
    assert s.dim() == 0 and float(s) == 0.0
