"""The PESQ back end's three forms (pesq.hip, pesq::back_waves): 8 waves per utterance for
batches up to half a row per CU, 4 up to 2 rows per CU, 1 above.  The same ragged rows scored in
batches that select each form agree within 1e-5 (only the summation order of the band totals and
of the window L2 sum differs), and rows of each batch agree with the oracle (the CPU restatement
of the reference, pinned by tests/golden) within the PESQ tolerance of tests/test_gpu_parity.py.
STOI / ESTOI do not depend on the batch at all (bitwise).  The batch sizes assume MI355X's 256
CUs; on another part the forms shift, the assertions still hold."""
import numpy as np
import pytest
import torch

from oracle import pesq_oracle

pytestmark = pytest.mark.gpu
PESQ_TOL = 5e-3


@pytest.fixture(scope="module")
def rows():
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    B, L = 640, 32000
    c, n, _ = speech_like_pairs(B, L, 16000, seed=11, device="cuda")
    rng = np.random.default_rng(11)
    lens = rng.integers(6000, L + 1, size=B)
    lens[::7] = L
    return c, n, torch.as_tensor(lens, dtype=torch.int32)


def test_back_forms_agree(rows):
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    c, n, lens = rows
    m = PESQ_STOI(16000, use_gpu=True)
    pick = torch.arange(0, 640, 37, device="cuda")  # 18 rows
    out = {}
    for B in (640, 300, 18):  # 1-wave, 4-wave, 8-wave form on 256 CUs
        idx = pick if B == 18 else torch.arange(B, device="cuda")
        mos, s, e = m.scores(c[idx].contiguous(), n[idx].contiguous(), lengths=lens[idx.cpu()])
        keep = pick[pick < B]
        pos = keep if B != 18 else torch.arange(18, device="cuda")
        out[B] = [t[pos].cpu().numpy() for t in (mos, s, e)]
    common = int((pick < 300).sum())
    for B in (300, 18):
        np.testing.assert_allclose(out[B][0][:common], out[640][0][:common], rtol=0, atol=1e-5)
        np.testing.assert_array_equal(out[B][1][:common], out[640][1][:common])
        np.testing.assert_array_equal(out[B][2][:common], out[640][2][:common])
    # a few rows against the oracle, each row alone (its own length)
    cc, nn, ll = c[pick[:4]].cpu().numpy(), n[pick[:4]].cpu().numpy(), lens[pick[:4].cpu()].numpy()
    want = np.array([pesq_oracle.pesq(cc[i:i + 1, :ll[i]], nn[i:i + 1, :ll[i]])[0] for i in range(4)])
    for B in (640, 300, 18):
        np.testing.assert_allclose(out[B][0][:4], want, rtol=0, atol=PESQ_TOL)
