"""GPU parity: the HIP engine (through the C-ABI, via the drop-in API) vs the reference's
golden vectors and the oracle.  Tolerances: PESQ +-5e-3 (the reference's own CPU-vs-GPU
bound, tests/test_cuda.py:23), STOI/ESTOI +-5e-4 (its pystoi bound, test_stoi.py:24-25);
intermediates relative.  The achieved deviations are far below."""
import numpy as np
import pytest
import torch

from tests.conftest import PESQ_CASES, STOI_CASES, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from fast_speech_enhancement_metrics_amd import _native
    _native.load()
    return torch.device("cuda:0")


def test_native_library_is_loaded(dev):
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    assert lib.fsem_version() >= 1


@pytest.mark.parametrize("name", PESQ_CASES)
def test_pesq_gpu_matches_reference(dev, name):
    from fast_speech_enhancement_metrics_amd import PESQ
    g = load_golden(name)
    res = PESQ(16000, use_gpu=True)(torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]))
    mos = np.array([d["PESQ"] for d in res])
    print(name, "max |dPESQ| vs reference:", np.abs(mos - g["pesq"]).max())
    np.testing.assert_allclose(mos, g["pesq"], atol=5e-3, rtol=0)


@pytest.mark.parametrize("name", ["pesq_3s", "pesq_ragged", "pesq_wide"])
def test_pesq_front_bark_matches_reference(dev, name):
    from fast_speech_enhancement_metrics_amd import _native
    g = load_golden(name)
    lib = _native.load()
    c = torch.from_numpy(g["clean_f"]).to(dev)
    n = torch.from_numpy(g["noisy_f"]).to(dev)
    B, L = c.shape
    c = torch.nn.functional.pad(c, (0, (-L) % 4)).contiguous()  # rows readable to ceil4(L)
    n = torch.nn.functional.pad(n, (0, (-L) % 4)).contiguous()
    ld = c.shape[1]
    F = lib.fsem_pesq_frames(L)
    bark = torch.empty(2 * B, 49, (F + 31) // 32 * 32, device=dev)  # band-major, rows padded to 32 frames
    power = torch.empty(2 * B, device=dev)
    ws = _native.workspace(lib.fsem_pesq_front_workspace_bytes(B, L), dev)
    _native.check(lib.fsem_pesq_front_f32(c.data_ptr(), n.data_ptr(), B, L, ld, None, bark.data_ptr(), power.data_ptr(),
                                          ws.data_ptr(), ws.numel(), _native.stream_handle(dev)), "front")
    torch.cuda.synchronize()
    p = power.double().cpu().numpy() / (L + 5120) / 1.04684
    # golden bark is after equalize_ranges + level alignment: scale = 1e7 / power of the raw signal
    scaled = bark[:, :, :F].transpose(1, 2).double().cpu().numpy() * (1e7 / p)[:, None, None]
    ref = g["bark"].astype(np.float64)
    rel = np.abs(scaled - ref).max() / np.abs(ref).max()
    print(name, "bark rel err", rel)
    assert rel < 5e-3
    # level-alignment scale sqrt(1e7 / power) (PESQ.py:100) vs the reference's
    m = np.maximum(np.abs(g["clean_f"]).max(1), np.abs(g["noisy_f"]).max(1))
    scale = np.sqrt(1e7 / p) * np.concatenate([m, m])
    np.testing.assert_allclose(scale, g["level_scale"], rtol=3e-3)


@pytest.mark.parametrize("name", STOI_CASES)
def test_stoi_gpu_matches_reference(dev, name):
    from fast_speech_enhancement_metrics_amd import STOI
    g = load_golden(name)
    res = STOI(int(g["sample_rate"]), use_gpu=True)(torch.from_numpy(g["clean_f"]), torch.from_numpy(g["noisy_f"]))
    s = np.array([d["STOI"] for d in res])
    e = np.array([d["ESTOI"] for d in res])
    print(name, "max |dSTOI|", np.abs(s - g["stoi"]).max(), "max |dESTOI|", np.abs(e - g["estoi"]).max())
    np.testing.assert_allclose(s, g["stoi"], atol=5e-4, rtol=0)
    np.testing.assert_allclose(e, g["estoi"], atol=5e-4, rtol=0)


def test_stoi_tob_matches_reference(dev):
    from fast_speech_enhancement_metrics_amd import _native
    g = load_golden("stoi_10k")
    lib = _native.load()
    c = torch.from_numpy(g["clean_f"]).to(dev)
    n = torch.from_numpy(g["noisy_f"]).to(dev)
    B, L = c.shape
    NV = (L - 256) // 128 + 1
    tmax = NV - 2
    kept = torch.empty(B, dtype=torch.int32, device=dev)
    tob = torch.zeros(2 * B, 15, tmax, device=dev)
    ws = _native.workspace(lib.fsem_stoi_workspace_bytes(B, L, 10000), dev)
    _native.check(lib.fsem_stoi_tob_f32(c.data_ptr(), n.data_ptr(), B, L, L, kept.data_ptr(), tob.data_ptr(), tmax,
                                        ws.data_ptr(), ws.numel(), _native.stream_handle(dev)), "tob")
    torch.cuda.synchronize()
    assert kept.cpu().numpy().tolist() == g["kept"].tolist()
    tob = tob.cpu().numpy()
    for b in range(B):
        T = int(g["kept"][b]) - 2
        for sig in (b, B + b):
            ref = g["tob"][sig][:, :T]
            err = np.abs(tob[sig][:, :T] - ref).max() / np.abs(ref).max()
            assert err < 1e-4, (b, sig, err)


def test_resample_gpu_matches_reference(dev):
    from fast_speech_enhancement_metrics_amd.resample import Resample
    g = load_golden("stoi_16k")
    out = Resample(16000, 10000).to(dev)(torch.from_numpy(g["clean_f"]).to(dev)).cpu().numpy()
    assert out.shape == g["x10_clean"].shape
    np.testing.assert_allclose(out, g["x10_clean"], atol=2e-6, rtol=0)


def test_device_parity_10s(dev):
    """tests/test_cuda.py:8-23 analogue: CPU mode vs GPU mode within 5e-3, 10 s @16 kHz."""
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    c, n, _ = speech_like_pairs(6, 160000, seed=123, snr_low=0, snr_high=40)
    for cls in (PESQ, STOI):
        cpu = cls(16000, use_gpu=False)(c, n)
        gpu = cls(16000, use_gpu=True)(c, n)
        for a, b in zip(cpu, gpu):
            for k in a:
                assert a[k] == pytest.approx(b[k], abs=5e-3), (cls.__name__, k, a[k], b[k])


def test_high_vs_low_snr(dev):
    """tests/test_high_vs_low_snr.py analogue on the GPU path."""
    from fast_speech_enhancement_metrics_amd import PESQ, STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    ch, nh, _ = speech_like_pairs(4, 64000, seed=7, snr_low=10, snr_high=10)
    cl, nl, _ = speech_like_pairs(4, 64000, seed=7, snr_low=-5, snr_high=-5)
    for cls in (PESQ, STOI):
        m = cls(16000, use_gpu=True)
        hi, lo = m(ch, nh), m(cl, nl)
        for a, b in zip(hi, lo):
            for k in a:
                assert a[k] > b[k], (cls.__name__, k)
