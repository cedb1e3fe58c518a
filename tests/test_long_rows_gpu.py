"""Long utterances: 5-minute rows against the oracle (the CPU restatement of the reference,
pinned by tests/golden) -- many segments per row in every kernel, the PESQ back end's multi-wave
form, STOI's segment blocks -- and a 1-hour pair through the joint entry checked by properties
(identical signals: PESQ at the ceiling, STOI / ESTOI = 1; a ragged copy of the same pair gives
the same scores for the full-length row)."""
import warnings

import numpy as np
import pytest
import torch

from oracle import pesq_oracle, stoi_oracle

pytestmark = pytest.mark.gpu
PESQ_TOL, STOI_TOL = 5e-3, 5e-4


def test_five_minute_rows_vs_oracle():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    L = 300 * 16000
    c, n, _ = speech_like_pairs(2, L, 16000, seed=21, device="cuda")
    lens = torch.tensor([L, L - 1234567], dtype=torch.int32)
    mos, s, e = (t.cpu().numpy() for t in PESQ_STOI(16000, use_gpu=True).scores(c, n, lengths=lens))
    cc, nn = c.cpu().numpy(), n.cpu().numpy()
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        for b in range(2):
            k = int(lens[b])
            op = pesq_oracle.pesq(cc[b:b + 1, :k], nn[b:b + 1, :k])[0]
            os_, oe = stoi_oracle.stoi(cc[b:b + 1, :k], nn[b:b + 1, :k], 16000)
            assert abs(mos[b] - op) < PESQ_TOL, (b, mos[b], op)
            assert abs(s[b] - os_[0]) < STOI_TOL and abs(e[b] - oe[0]) < STOI_TOL, (b, s[b], os_, e[b], oe)


def test_one_hour_pair_properties():
    from fast_speech_enhancement_metrics_amd import PESQ_STOI
    from fast_speech_enhancement_metrics_amd.synthetic import speech_like_pairs
    L = 3600 * 16000
    c, n, _ = speech_like_pairs(1, L, 16000, seed=22, device="cuda")
    m = PESQ_STOI(16000, use_gpu=True)
    mos, s, e = (t.cpu().numpy() for t in m.scores(torch.cat([c, c]), torch.cat([c, n])))
    assert mos[0] > 4.6 and abs(s[0] - 1) < 1e-5 and abs(e[0] - 1) < 1e-5, (mos, s, e)
    assert np.isfinite(mos).all() and np.isfinite(s).all() and np.isfinite(e).all()
    assert 1.0 <= mos[1] <= 4.65 and 0 < s[1] < 1 and 0 < e[1] < 1
    # the same pair as a ragged row (a shorter companion row): same scores
    lens = torch.tensor([L, L // 3], dtype=torch.int32)
    mos2, s2, e2 = (t.cpu().numpy() for t in m.scores(torch.cat([c, c]), torch.cat([n, n]), lengths=lens))
    np.testing.assert_allclose([mos2[0], s2[0], e2[0]], [mos[1], s[1], e[1]], rtol=0, atol=1e-5)
