"""Edge inputs against the reference itself (tests/golden/edges_16k.npz, tone_probe_10k.npz; VERDICT r2
item 1): DC offsets, extreme common scales, full-scale tones.  Each golden holds the reference run
twice -- PESQ with two admissible float32 FIR evaluation orders, STOI/ESTOI with torch seeds 0 and
1 -- and the bar for the engine is BASELINE's +-0.01 widened by that spread where the reference's
own result moves with evaluation order or seed (the domain limits documented in include/fsem.h).
"""
import numpy as np
import pytest
import torch

from tests.conftest import edge_inputs, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def edges():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return load_golden("edges_16k")


def _engine(c, n):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    p, s, e = PESQ_STOI(16000, use_gpu=True).scores(c.cuda(), n.cuda())
    return p.cpu().double().numpy(), s.cpu().double().numpy(), e.cpu().double().numpy()


def _bar(a, b, floor=0.01):
    """BASELINE's +-0.01, or the spread of the reference's two runs where that is larger."""
    spread = np.nanmax(np.abs(np.asarray(a) - np.asarray(b))) if np.isfinite(a).any() else 0.0
    return max(floor, 2 * spread)


@pytest.mark.parametrize("name", ["dc100_clean", "dc100_both", "dc1000_both", "scale_1e-15", "scale_1e18"])
def test_pesq_edges_match_reference(edges, name):
    c, n = edge_inputs(edges, name)
    p, _, _ = _engine(c, n)
    ref, alt = edges[name + "_pesq"], edges[name + "_pesq_f64fir"]
    bar = _bar(ref, alt)
    print(name, "PESQ engine", p, "reference", ref, "alt order", alt, "bar", bar)
    assert np.isfinite(p).all()
    np.testing.assert_allclose(p, ref, atol=bar, rtol=0)


@pytest.mark.parametrize("name", ["dc100_clean", "dc100_both", "dc1000_both"])
def test_stoi_edges_match_reference(edges, name):
    c, n = edge_inputs(edges, name)
    _, s, e = _engine(c, n)
    for got, key in ((s, "_stoi"), (e, "_estoi")):
        ref, alt = edges[name + key], edges[name + key + "_seed1"]
        bar = _bar(ref, alt, floor=5e-4)
        print(name, key, "engine", got, "reference", ref, "bar", bar)
        np.testing.assert_allclose(got, ref, atol=bar, rtol=0)


def test_stoi_tiny_scale_is_seed_noise_in_the_reference(edges):
    """At 1e-15 the reference's STOI/ESTOI are its 1e-12 * randn term (STOI.py:116): seed 0 and 1
    differ by ~1e-2 around 0, so no implementation can be pinned closer; the engine gives scores
    within that noise band of 0, never NaN."""
    name = "scale_1e-15"
    c, n = edge_inputs(edges, name)
    _, s, e = _engine(c, n)
    for got, key in ((s, "_stoi"), (e, "_estoi")):
        ref, alt = edges[name + key], edges[name + key + "_seed1"]
        band = max(np.abs(ref).max(), np.abs(alt).max(), np.abs(ref - alt).max())
        print(name, key, "engine", got, "reference seeds", ref, alt)
        assert band < 0.05
        assert np.isfinite(got).all() and np.abs(got).max() <= max(3 * band, 0.05)


def test_stoi_huge_scale(edges):
    """At 1e18 the reference's float32 power spectrum overflows (|X|^2 > 3.4e38): STOI NaN in every
    row.  The engine reports what it computes; the test records both (documented domain limit)."""
    name = "scale_1e18"
    c, n = edge_inputs(edges, name)
    _, s, e = _engine(c, n)
    print(name, "engine", s, e, "reference", edges[name + "_stoi"], edges[name + "_estoi"])
    assert np.isnan(edges[name + "_stoi"]).all()


def test_tone_probe_matches_reference():
    g = load_golden("tone_probe_10k")
    from fast_speech_enhancement_metrics_amd import STOI
    s, e = STOI(10000, use_gpu=True).scores(torch.from_numpy(g["clean_f"]).cuda(), torch.from_numpy(g["noisy_f"]).cuda())
    s, e = s.cpu().double().numpy(), e.cpu().double().numpy()
    print("tone probe STOI", s, g["stoi"], "ESTOI", e, g["estoi"])
    np.testing.assert_allclose(s, g["stoi"], atol=0.01, rtol=0)
    np.testing.assert_allclose(e, g["estoi"], atol=0.01, rtol=0)
