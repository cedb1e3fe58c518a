"""Pin the oracle (CPU restatement) against vectors produced by the reference itself.

Golden vectors: tests/golden/*.npz, made by tests/golden/make_golden.py, which runs the
reference's own fast_se_metrics.PESQ / STOI (torchaudio restated, see oracle/ta_shim).
"""
import numpy as np

from oracle import pesq_oracle, stoi_oracle, ta


def test_oracle_pesq_matches_reference(pesq_golden):
    g = pesq_golden
    inter = {}
    mos = pesq_oracle.pesq(g["clean_f"], g["noisy_f"], inter)
    # fp32 10th-order direct-form IIR noise in the reference itself is ~1e-4 in MOS
    np.testing.assert_allclose(mos, g["pesq"], atol=2e-3, rtol=0)
    bark = np.concatenate([inter["bark_clean"], inter["bark_noisy"]])
    assert bark.shape == g["bark"].shape
    err = np.abs(bark - g["bark"]).max() / np.abs(g["bark"]).max()
    assert err < 5e-3  # level power carries the reference's fp32 direct-form IIR noise (~1e-3)


def test_oracle_level_scale(pesq_golden):
    g = pesq_golden
    c, n = pesq_oracle.equalize_ranges(g["clean_f"], g["noisy_f"])
    s = np.concatenate([c, n])
    scale = np.sqrt(1e7 / pesq_oracle.level_power(s)[:, 0])
    np.testing.assert_allclose(scale, g["level_scale"], rtol=3e-3)


def test_oracle_stoi_matches_reference(stoi_golden):
    g = stoi_golden
    inter = []
    s, e = stoi_oracle.stoi(g["clean_f"], g["noisy_f"], int(g["sample_rate"]), inter)
    np.testing.assert_allclose(s, g["stoi"], atol=1e-5, rtol=0)
    np.testing.assert_allclose(e, g["estoi"], atol=1e-5, rtol=0)
    assert [d["kept"] for d in inter] == list(g["kept"])
    B = s.shape[0]
    for b in range(B):
        T = inter[b]["tob_clean"].shape[1]
        ref_c = g["tob"][b][:, :T]
        ref_n = g["tob"][B + b][:, :T]
        scale = np.abs(ref_c).max()
        assert np.abs(inter[b]["tob_clean"] - ref_c).max() / scale < 1e-5
        assert np.abs(inter[b]["tob_noisy"] - ref_n).max() / scale < 1e-5


def test_oracle_resample_matches_reference():
    from tests.conftest import load_golden
    g = load_golden("stoi_16k")
    x10 = ta.resample(g["clean_f"], 16000, 10000)
    assert x10.shape == g["x10_clean"].shape
    np.testing.assert_allclose(x10, g["x10_clean"], atol=2e-6, rtol=0)


def test_resample_kernel_shape():
    k, width, orig, new = ta.sinc_resample_kernel(16000, 10000)
    assert (orig, new, width) == (8, 5, 10) and k.shape == (5, 28)
    k2, w2, o2, n2 = ta.sinc_resample_kernel(8000, 16000)
    assert (o2, n2) == (1, 2) and k2.shape == (2, 2 * w2 + 1)
