"""The resampler's two GPU forms (csrc/resample.hip): the direct form (float4-aligned rows, the
8->16, 8->10 and 48->16 kHz pairs) and the LDS-tiled form (everything else) against the oracle's
torchaudio restatement (oracle/ta.py, pinned by the x10 golden of tests/golden), and bitwise
against each other -- both keep resample_at's tap order.  Lengths cover row tails that end inside a
float4 chunk, rows shorter than the filter, and a length of one sample."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import ta

pytestmark = pytest.mark.gpu
RATES = [(8000, 16000), (8000, 10000), (48000, 16000), (16000, 10000)]
LENGTHS = [1, 7, 37, 4000, 4001, 4003, 24000]


def _resample(lib, x, ld_in, orig, new):
    """fsem_resample_f32 over the first n columns of x (rows of ld_in floats)."""
    from fast_speech_enhancement_metrics_amd import _native
    rows = x.shape[0]
    n = x.shape[1]
    buf = torch.zeros(rows, ld_in, dtype=torch.float32, device="cuda")
    buf[:, :n] = x
    n_out = lib.fsem_resample_length(n, orig, new)
    out = torch.full((rows, n_out), float("nan"), dtype=torch.float32, device="cuda")
    _native.check(lib.fsem_resample_f32(ctypes.c_void_p(buf.data_ptr()), rows, n, ld_in,
                                        ctypes.c_void_p(out.data_ptr()), n_out, orig, new,
                                        ctypes.c_void_p(_native.stream_handle())), "resample")
    return out


@pytest.mark.parametrize("orig,new", RATES)
@pytest.mark.parametrize("n", LENGTHS)
def test_resample_forms_vs_oracle_and_each_other(orig, new, n):
    from fast_speech_enhancement_metrics_amd import _native
    lib = _native.load()
    rng = np.random.default_rng(n * 7 + orig + new)
    x = rng.standard_normal((3, n)).astype(np.float32)
    xt = torch.from_numpy(x).cuda()
    aligned = _resample(lib, xt, (n + 3) // 4 * 4, orig, new)   # direct form for the listed pairs
    tiled = _resample(lib, xt, (n + 3) // 4 * 4 + 1, orig, new)  # odd row stride: tiled form
    torch.cuda.synchronize()
    a, t = aligned.cpu().numpy(), tiled.cpu().numpy()
    ref = ta.resample(x, orig, new)
    assert a.shape == ref.shape
    np.testing.assert_array_equal(a, t)
    np.testing.assert_allclose(a, ref, atol=2e-6 * max(1.0, np.abs(ref).max()), rtol=0)


@pytest.mark.parametrize("orig,new", RATES)
@pytest.mark.parametrize("n", [4000, 4003])
def test_resample_rows_ragged(orig, new, n):
    """fsem_resample_rows_f32 (Resample.forward with lengths): each row equals the oracle on the row
    alone, the rest of the row is zero, and both forms agree bitwise."""
    from fast_speech_enhancement_metrics_amd import _native
    from fast_speech_enhancement_metrics_amd.resample import Resample
    rng = np.random.default_rng(n + orig)
    lens = np.array([n, 1, 7, 37, n - 1, n // 2, 0, 1001], dtype=np.int32)
    x = rng.standard_normal((len(lens), n)).astype(np.float32)  # tails are NOT zero
    xt = torch.from_numpy(x).cuda()
    out = Resample(orig, new).cuda()(xt, torch.from_numpy(lens).cuda()).cpu().numpy()
    # the same rows with an odd stride go through the tiled form
    lib = _native.load()
    ld = n + 1 if (n + 1) % 4 else n + 2  # not a multiple of 4
    buf = torch.zeros(len(lens), ld, device="cuda")
    buf[:, :n] = xt
    n_out = lib.fsem_resample_length(n, orig, new)
    tiled = torch.full((len(lens), n_out), float("nan"), device="cuda")
    _native.check(lib.fsem_resample_rows_f32(buf.data_ptr(), len(lens), n, ld,
                                             torch.from_numpy(lens).cuda().data_ptr(), tiled.data_ptr(), n_out,
                                             orig, new, _native.stream_handle()), "resample rows")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out, tiled.cpu().numpy())
    for r, ln in enumerate(lens):
        k = lib.fsem_resample_length(int(ln), orig, new)
        if ln:
            ref = ta.resample(x[r:r + 1, :ln], orig, new)[0]
            np.testing.assert_allclose(out[r, :k], ref, atol=2e-6 * max(1.0, np.abs(ref).max()), rtol=0)
        assert (out[r, k:] == 0).all(), r
